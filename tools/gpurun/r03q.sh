# round-3 pass Q: A/B HEAD vs HEAD + global (not flat) candidate loads at 8,192; fused wave timeline with the slowest waves
export TMPDIR=/tmp
O=gpurun_out/r03q
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab.txt 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 > $O/timeline_8192.txt 2>&1 || exit $?
cat $O/ab.txt $O/timeline_8192.txt
