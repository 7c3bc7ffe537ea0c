export TMPDIR=/tmp
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_stamps.so timeout -k 10 300 python tests/_stamps_report.py > gpurun_out/stamps.log 2>&1 || exit $?
cat gpurun_out/stamps.log
