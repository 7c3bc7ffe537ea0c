export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/q/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/q/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q/bench.json 2>gpurun_out/q/bench.err || exit $?
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_stamps.so timeout -k 10 300 python tests/_stamps_report.py > gpurun_out/q/stamps.log 2>&1 || exit $?
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/q/pmc -o write --output-format csv -- $B > gpurun_out/q/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d gpurun_out/q/pmc -o lds --output-format csv -- $B > gpurun_out/q/pmc_lds.log 2>&1 || exit $?
echo QDONE
