# round-3 pass M: no flat loads (global hull pointers, value-selected hull frames): full GPU suite, bench lines, EPA stamps
export TMPDIR=/tmp
O=gpurun_out/r03m
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_65536.json 2> $O/bench_65536.err || exit $?
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_epastamps.so timeout -k 10 200 python tools/dev/epa_stamps.py 8192 fused > $O/epa_fused.txt 2>&1 || exit $?
echo R03M_DONE
