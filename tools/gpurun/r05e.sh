# round 5: the GPU suite after the PGS env order was dropped (round 4's dispatch and contact update, the QCQP's
# hardware reciprocals kept) and the fused path's compact contact counts; PGS bench lines; per-step PMC traffic at
# 65,536 envs (the write figure); the 65,536 bench line
export TMPDIR=/tmp
O=gpurun_out/r05e
rm -rf $O; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline --steps 100 --contact-steps 0 > $O/pgs_$r.json 2> $O/pgs_$r.err || exit $?
done
n=65536
B="python bench.py --total-envs $n --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
P=$O/pmc_fused_$n
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
python tools/gpurun/pmc_step_traffic.py $P $n fused newton 40 5 $O/r05_pmc_step_fused_newton_$n.json > $P.traffic.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
echo R05E_DONE
