# round-2 measurement set (writes gpurun_out/r02/*): GPU tests, smoke, bench line (Newton, fused step),
# kernel trace + stats, PMC traffic / SQ counters of the fused kernel, per-shard-size rates (fused and
# split), PGS bench line and trace.
export TMPDIR=/tmp
O=gpurun_out/r02
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
B="python bench.py --steps 4 --warmup 60 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o fetch --output-format csv -- $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- $B > $O/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc -o sq --output-format csv -- $B > $O/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc -o misc --output-format csv -- $B > $O/pmc_misc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/pmc -o sqc --output-format csv -- $B > $O/pmc_sqc.log 2>&1 || exit $?
python tests/_pmc_traffic.py $O/pmc 65536 $O/pmc_traffic_fused.json 1 fused > $O/pmc_traffic.log 2>&1 || exit $?
python tests/_pmc_report.py $O/pmc > $O/pmc_report.txt 2>&1 || exit $?
python tests/_trace_report.py $O/trace > $O/trace_report.txt 2>&1 || exit $?
lscpu > $O/lscpu.txt 2>&1; nproc > $O/nproc.txt; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> $O/nproc.txt
for n in 65536 32768 16384 8192; do
  for f in 1 0; do
    SO100_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/shard_f${f}_$n.json 2>>$O/shard.err || exit $?
  done
done
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o bench_pgs --output-format csv -- python bench.py --solver pgs --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_pgs.log 2>&1 || exit $?
echo ROUND2DONE
