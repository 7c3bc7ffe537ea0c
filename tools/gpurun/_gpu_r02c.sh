# fused-kernel A/B (writes gpurun_out/r02c/*): fused parity tests, then bench at the 1-GPU and the 8-GPU
# shard sizes for the in-tree build (fused, 3 waves/SIMD), variants fused2 (2 waves/SIMD) and noids (no
# per-substep id laundering), and the split path (SO100_FUSED=0).
export TMPDIR=/tmp
O=gpurun_out/r02c
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "fused or step_mode or chunking" > $O/pytest_fused.log 2>&1 || exit $?
for n in 65536 8192; do
  B="python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10"
  timeout -k 10 200 $B > $O/fused_$n.json 2>$O/err || exit $?
  for v in fused2 noids; do SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 $B > $O/${v}_$n.json 2>$O/err || exit $?; done
  SO100_FUSED=0 timeout -k 10 200 $B > $O/split_$n.json 2>$O/err || exit $?
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f); done
echo R02CDONE
