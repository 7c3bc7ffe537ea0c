# round 4: the deep-fold tests under the ensemble gate, the chunking test, the overflow outliers
export TMPDIR=/tmp
O=gpurun_out/r04b
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/dev/overflow_outliers.py newton 1 > $O/outliers_newton1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dev/overflow_outliers.py pgs 1 > $O/outliers_pgs1.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rA --timeout 400 --timeout-method thread -s \
  -k "chunking or arm_contact or overflow or self_collision or base_contact or pad_link" > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log

bash tools/gpurun/abtree.sh $O/ab r03 65536 3 150 > $O/ab_65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab r03 8192 3 300 > $O/ab_8192.txt 2>&1 || exit $?
echo R04B_AB_DONE
