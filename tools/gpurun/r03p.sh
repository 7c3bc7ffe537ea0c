# round-3 pass P: A/B HEAD vs no-flat-loads only (nosat) vs + box SAT (current), 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r03p
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O/a $V/libso100_hip_base.so $V/libso100_hip_nosat.so 8192 3 > $O/ab_base_nosat.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/b $V/libso100_hip_nosat.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab_nosat_sat.txt 2>&1 || exit $?
cat $O/ab_*.txt
