# round 5: repeat runs of the default bench line and the 8,192-env shard on the closing tree (run-to-run spread)
export TMPDIR=/tmp
O=gpurun_out/r05w
rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
  timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192_$r.json 2> $O/bench_8192_$r.err || exit $?
done
echo R05W_DONE
