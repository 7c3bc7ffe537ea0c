# round 4: the overflow outliers in detail; A/B of the overflow paths and the collision reorder
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04c}
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/dev/overflow_outliers.py newton 1 > $O/outliers_newton1.log 2>&1 || exit $?
L=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O/ab_noovf $L/libso100_hip_head.so $L/libso100_hip_noovf.so 65536 3 > $O/ab_noovf_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab_noovf $L/libso100_hip_head.so $L/libso100_hip_noovf.so 8192 3 > $O/ab_noovf_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab_reorder $L/libso100_hip_head.so $L/libso100_hip_reorder.so 65536 3 > $O/ab_reorder_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab_reorder $L/libso100_hip_head.so $L/libso100_hip_reorder.so 8192 3 > $O/ab_reorder_8192.txt 2>&1 || exit $?
echo R04C_DONE
