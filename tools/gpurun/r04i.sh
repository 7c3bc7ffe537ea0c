# round 4: one Newton solve with the overflow paths vs two instantiations chosen per wave (same box, interleaved);
# the base / overflow deep-fold outliers in detail (states dumped for a CPU replay)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04i
rm -rf $O; mkdir -p $O
L=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O/ab $L/libso100_hip_onesolve.so $L/libso100_hip_twosolve.so 65536 3 > $O/ab_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab $L/libso100_hip_onesolve.so $L/libso100_hip_twosolve.so 8192 3 > $O/ab_8192.txt 2>&1 || exit $?
SO100_LIB=$L/libso100_hip_onesolve.so timeout -k 10 300 python -u tools/dev/overflow_outliers.py newton 0 $O/states_base.npz base > $O/outliers_base.log 2>&1 || exit $?
SO100_LIB=$L/libso100_hip_onesolve.so timeout -k 10 300 python -u tools/dev/overflow_outliers.py newton 0 $O/states_overflow.npz overflow > $O/outliers_overflow.log 2>&1 || exit $?
echo R04I_DONE
