# fused (heavy-first order, 12 waves/CU) vs split sweep (gpurun_out/r02f/*)
export TMPDIR=/tmp
O=gpurun_out/r02f
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "fused or step_mode or chunking or graph" > $O/pytest_fused.log 2>&1 || exit $?
for n in 65536 32768 16384 8192; do
  for f in 1 0; do
    SO100_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/f${f}_$n.json 2>$O/err || exit $?
  done
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f); done
echo R02FDONE
