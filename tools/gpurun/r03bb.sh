# DR scales / step counters re-read per substep in the fused kernel (SO100_FUSED_RELOAD=1: 3-wave spill slots 72 -> 60
# B/lane) vs the tree's build; Newton phase stamps (split solver kernel) at 8,192 envs on the current kernels
export TMPDIR=/tmp
O=gpurun_out/r03bb
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
L=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so
bash tools/gpurun/ab.sh $O/ab65536 $L $V/libso100_hip_reload1.so 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $L $V/libso100_hip_reload1.so 8192 3 > $O/ab8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/nstamps_8192.txt 2>&1 || exit $?
echo R03BB_DONE
