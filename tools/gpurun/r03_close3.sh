# round-3 closing set on the final kernels: GPU suite, smoke, bench lines (65,536 with the CPU baseline; the 2-, 4- and
# 8-GPU shard sizes; the split step at 65,536; PGS), rocprofv3 kernel traces of the bench commands, per-step PMC
# traffic (fused at every shard size, split at 65,536), the fused wave timeline at 8,192, host CPU facts
export TMPDIR=/tmp
O=gpurun_out/r03close3
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
for n in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --total-envs $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
SO100_FUSED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $O/bench_65536_split.json 2> $O/bench_65536_split.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --solver pgs --steps 200 > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
for cfg in "fused 65536" "split 65536" "fused 8192" "fused 16384" "fused 32768"; do
  set -- $cfg
  B="python bench.py --total-envs $2 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  P=$O/pmc_$1_$2
  if [ $1 = split ]; then export SO100_FUSED=0; else unset SO100_FUSED; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
  unset SO100_FUSED
  python tools/gpurun/pmc_step_traffic.py $P $2 $1 newton 40 5 $O/r03_pmc_step_$1_newton_$2.json > $P.traffic.log 2>&1 || exit $?
done
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 > $O/timeline_8192.txt 2>&1 || exit $?
lscpu > $O/lscpu.txt 2>&1; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())" > $O/affinity.txt
echo R03CLOSE3_DONE
