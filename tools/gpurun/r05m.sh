# round 5: the convex broadphase's stages in the stage stamps (variant sstampsbroad: slot "Euler" = the sphere table and
# tests, slot "S7 + record" = the OBB stage and lists (+ S7), slot "S3b" = the narrowphase rounds), 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05m
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 65536 8192; do
  SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstampsbroad.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $n > $O/sstampsbroad_$n.txt 2>&1 || exit $?
done
echo R05M_DONE
