# (1) DR scales / step counters re-read per substep in the fused kernel (SO100_FUSED_RELOAD=1: 3-wave spill slots
# 72 -> 60 B/lane); (2) supports of hulls of <= 16 vertices from register-held vertices (SO100_SMALL_HULL_REG=1):
# GPU suite on (2), A/Bs of both against the tree's build; Newton phase stamps at 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r03bb
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
L=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so
SO100_LIB=$V/libso100_hip_sreg.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu_sreg.log 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/sreg65536 $L $V/libso100_hip_sreg.so 65536 3 > $O/ab_sreg_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/sreg8192 $L $V/libso100_hip_sreg.so 8192 3 > $O/ab_sreg_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/rl65536 $L $V/libso100_hip_reload1.so 65536 3 > $O/ab_reload_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/rl8192 $L $V/libso100_hip_reload1.so 8192 3 > $O/ab_reload_8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/nstamps_8192.txt 2>&1 || exit $?
echo R03BB_DONE
