export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_base_$i.log 2>&1 || exit $?
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_noslp.so timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_noslp_$i.log 2>&1 || exit $?
done
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_stamps.so timeout -k 10 300 python tests/_stamps_report.py > gpurun_out/stamps.log 2>&1 || exit $?
for f in gpurun_out/ab_*.log; do echo $f $(grep -o '"value": [0-9.]*' $f); done
