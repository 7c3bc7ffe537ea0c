# round-3 pass B: the parity suite after the conditioning floor and the per-substep arm-contact tests
export TMPDIR=/tmp
O=gpurun_out/r03b
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
echo R03B_DONE
