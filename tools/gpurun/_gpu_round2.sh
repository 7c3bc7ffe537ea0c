# round-2 measurement set (writes gpurun_out/r02/*): GPU tests, smoke, the bench line (65,536 envs on 1 GPU:
# Newton, split step), its kernel trace + PMC traffic / SQ counters of the Newton kernel; the 8-GPU shard
# (8,192 envs: fused step) likewise; per-shard-size rates in both step modes; PGS bench line and trace.
export TMPDIR=/tmp
O=gpurun_out/r02
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
for cfg in "split 65536 16384 4 newton" "fused 8192 8192 1 fused"; do
  set -- $cfg
  B="python bench.py --total-envs $2 --steps 4 --warmup 60 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
  P=$O/pmc_$1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $P -o misc --output-format csv -- $B > $P.misc.log 2>&1 || exit $?
  python tools/gpurun/_pmc_traffic.py $P $3 $O/pmc_traffic_$5.json $4 $5 > $P.traffic.log 2>&1 || exit $?
  python tools/gpurun/_pmc_report.py $P > $O/pmc_report_$1.txt 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
python tools/gpurun/_trace_report.py $O/trace > $O/trace_report.txt 2>&1 || exit $?
python tools/gpurun/_trace_report.py $O/trace_fused >> $O/trace_report.txt 2>&1 || exit $?
lscpu > $O/lscpu.txt 2>&1; nproc > $O/nproc.txt; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> $O/nproc.txt
for n in 65536 32768 16384 8192; do
  for f in 1 0; do
    SO100_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/shard_f${f}_$n.json 2>>$O/shard.err || exit $?
  done
done
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o bench_pgs --output-format csv -- python bench.py --solver pgs --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_pgs.log 2>&1 || exit $?
echo ROUND2DONE
