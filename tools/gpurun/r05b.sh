# round 5: the GPU suite on the f2 kernels (table pairs at the minimum penetration) and the unconditional deep-fold
# floor; a same-box A/B of the round-4 tree (abtree/r04) against this tree at 65,536 and 8,192 envs (the f2 cost);
# bench lines; the fused kernel's wave timeline at 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05b
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpurun/abtree.sh $O/ab65536 r04 65536 2 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r04 8192 2 300 > $O/ab8192.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 $O/timeline_8192.npz > $O/timeline_8192.txt 2>&1 || exit $?
echo R05B_DONE
