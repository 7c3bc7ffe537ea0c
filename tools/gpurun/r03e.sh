# round-3 pass E: PGS outliers (substep walk), EPA vs MPR at the 8-GPU shard (bench + wave timeline)
export TMPDIR=/tmp
O=gpurun_out/r03e
rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/dev/tf_outlier.py mpr pgs epa $O/mpr_pgs_epa.npz > $O/outlier_mpr_pgs_epa.txt 2>&1 || exit $?
BY_QACC=1 timeout -k 10 300 python tools/dev/tf_outlier.py heavy pgs epa $O/heavy_pgs.npz > $O/outlier_heavy_pgs.txt 2>&1 || exit $?
for c in epa mpr; do
  timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline --convex $c > $O/bench_8192_$c.json 2> $O/bench_8192_$c.err || exit $?
  CONVEX=$c SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 > $O/timeline_8192_$c.txt 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --convex mpr > $O/bench_65536_mpr.json 2> $O/bench_65536_mpr.err || exit $?
echo R03E_DONE
