# round 4: the deep-fold / overflow parity tests (the ensemble gate with the FMA-contracted fp32 floor)
export TMPDIR=/tmp
O=gpurun_out/r04h
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rA --timeout 400 --timeout-method thread -s \
  -k "arm_contact or overflow or self_collision or base_contact or pad_link or cube_on_base" > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
echo R04H_DONE
