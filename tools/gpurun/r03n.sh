# round-3 pass N: fused wave timeline at 8,192 envs (EPA), A/B of the current build vs itself (noise floor)
export TMPDIR=/tmp
O=gpurun_out/r03n
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 > $O/timeline_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O gym-so100-c_amd/gym_so100/_lib/libso100_hip.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab.txt 2>&1 || exit $?
cat $O/timeline_8192.txt $O/ab.txt
