# stage phase stamps with the convex narrowphase compiled out after the broadphase (the broadphase's own cost)
export TMPDIR=/tmp
O=gpurun_out/r03y
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstampsbroad.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/sstampsbroad_8192.txt 2>&1 || exit $?
echo R03Y_DONE
