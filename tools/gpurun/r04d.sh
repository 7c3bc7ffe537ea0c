# round 4: r04c (pre-marker tree in abtree/cur: outliers + A/B of the overflow paths and the collision reorder),
# then the marker tree's EE parity tests
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd abtree/cur && OUT=$R/gpurun_out/r04c bash tools/gpurun/r04c.sh) || exit $?
mkdir -p gpurun_out/r04d
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "ee_weld or chunking or fused_step_matches" > gpurun_out/r04d/ee_tests.log 2>&1 || exit $?
echo R04D_DONE
