# round 6 closing measurements, part 2: the bench lines on the final kernels (quoting part 1's PMC files, now in
# profiles/): the default line (65,536 envs, CPU baseline), the shard sizes, configs[3] (GoalEnv 16,384), configs[4]
# (DR, the 8,192-env shard of 4 GPUs), PGS; the driver's window (--steps 20 --warmup 5) three times.
export TMPDIR=/tmp
O=gpurun_out/r06z
rm -rf $O; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
for n in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --total-envs $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
timeout -k 10 300 python bench.py --total-envs 16384 --task so100_goal > $O/bench_goal_16384.json 2> $O/bench_goal_16384.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --dr > $O/bench_dr_8192.json 2> $O/bench_dr_8192.err || exit $?
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$r.json 2> $O/drv_$r.err || exit $?
done
echo R06Z_DONE
