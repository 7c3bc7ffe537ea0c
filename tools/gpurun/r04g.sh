# round 4 closing measurements: the default bench line (65,536 envs + CPU baseline), the 8,192-env shard, PGS,
# rocprofv3 kernel stats, per-step PMC traffic at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r04g
rm -rf $O; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs.log 2>&1 || exit $?
for cfg in "fused 65536" "fused 8192"; do
  set -- $cfg
  B="python bench.py --total-envs $2 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  P=$O/pmc_$1_$2
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
  python tools/gpurun/pmc_step_traffic.py $P $2 $1 newton 40 5 $O/r04_pmc_step_$1_newton_$2.json > $P.traffic.log 2>&1 || exit $?
done
lscpu > $O/lscpu.txt 2>&1; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())" > $O/affinity.txt
echo R04G_DONE
