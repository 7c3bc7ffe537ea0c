# round 5: the fused 2-wave build in its own translation unit under the iterative-ILP scheduler (this tree) against
# HEAD 69f68a6's kernels (abtree/r05w): bitwise checks (product builds, fused vs split), same-box A/B at 8,192 and
# 65,536 envs; and PGS at 65,536 with every kernel under the iterative-ILP scheduler (variant sched_iterative-ilp)
export TMPDIR=/tmp
O=gpurun_out/r05q
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "product_builds or fused_step_matches_split or heavy_contact or step_parity_teacher or pool_contention" > $O/pytest.log 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05w 8192 3 300 > $O/ab8192.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab65536 r05w 65536 2 > $O/ab65536.txt 2>&1 || exit $?
P="python bench.py --solver pgs --no-cpu-baseline --steps 60 --contact-steps 0"
for r in 1 2; do
  timeout -k 10 200 $P > $O/pgs_base_$r.json 2> $O/pgs_base_$r.err || exit $?
  SO100_LIB=$V/libso100_hip_sched_iterative-ilp.so timeout -k 10 200 $P > $O/pgs_iter_$r.json 2> $O/pgs_iter_$r.err || exit $?
done
echo R05Q_DONE
