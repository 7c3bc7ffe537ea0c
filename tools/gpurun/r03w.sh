# re-entry check on HEAD: GPU suite, smoke, bench at 65,536 and at the 8-GPU shard
export TMPDIR=/tmp
O=gpurun_out/r03w
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline --steps 300 > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
echo R03W_DONE
# A/B: lane / env ids recomputed from v_mbcnt in the fused loop (SO100_LAUNDER_IDS=2) vs laundered copies (1)
V=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_ids1.so $V/libso100_hip_ids2.so 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_ids1.so $V/libso100_hip_ids2.so 8192 3 > $O/ab8192.txt 2>&1 || exit $?
echo AB_DONE
