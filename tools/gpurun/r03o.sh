# round-3 pass O: box-axis SAT prefilter before GJK, no flat loads: GPU suite, A/B vs HEAD at 8,192 / 65,536, EPA stamps
export TMPDIR=/tmp
O=gpurun_out/r03o
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpurun/ab.sh $O $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 65536 2 > $O/ab_65536.txt 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_epastamps.so timeout -k 10 200 python tools/dev/epa_stamps.py 8192 fused > $O/epa_fused.txt 2>&1 || exit $?
cat $O/ab_8192.txt $O/ab_65536.txt $O/epa_fused.txt
echo R03O_DONE
