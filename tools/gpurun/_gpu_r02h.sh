# GPU parity suite + bench line + fused/split per shard size on the current build (gpurun_out/r02h/*)
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02h}
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
for n in 65536 32768 16384 8192; do for f in 1 0; do
  SO100_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/shard_f${f}_$n.json 2>>$O/shard.err || exit $?
done; done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f); done
