# round-2 check after the fused kernel + auto mode (gpurun_out/r02e/*): full GPU suite, bench per shard size
export TMPDIR=/tmp
O=gpurun_out/r02e
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
for n in 65536 32768 16384 8192; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/bench_$n.json 2>$O/err || exit $?
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"step_mode": "[a-z]*"' $f); done
echo R02EDONE
