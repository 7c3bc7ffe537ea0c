# round-3 pass U: v_rcp / v_rsq in the contact, limit and frictionloss row setup, the dynamics Cholesky, Euler; the solimp power-2 impedance without powf (A/B vs HEAD)
export TMPDIR=/tmp
O=gpurun_out/r03u
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpurun/ab.sh $O/a $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/b $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 65536 2 > $O/ab_65536.txt 2>&1 || exit $?
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
cat $O/ab_*.txt
