# round-2 fused-kernel check (writes gpurun_out/r02b/*): new parity tests, then the full GPU suite, then
# bench at the 1-GPU and 8-GPU shard sizes: fused (default, 2 waves/SIMD), fused at 3 waves/SIMD (spilling
# variant), split (SO100_FUSED=0).
export TMPDIR=/tmp
O=gpurun_out/r02b
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "fused or step_mode" > $O/pytest_fused.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for n in 65536 8192; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/fused_$n.json 2>$O/err_f_$n || exit $?
  SO100_LIB=$V/libso100_hip_fused3.so timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/fused3_$n.json 2>$O/err_f3_$n || exit $?
  SO100_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/split_$n.json 2>$O/err_s_$n || exit $?
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f); done
echo R02BDONE
