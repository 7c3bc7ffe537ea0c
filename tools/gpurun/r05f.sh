# round 5: where the stage time goes on the current kernels: stage stamps (split path) with and without the box-box
# pairs split out (SO100_STAMP_BOXBOX: slot 0) at 65,536 and 8,192 envs; Newton stamps and the fused wave timeline
# at 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05f
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 65536 8192; do
  SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $n > $O/sstamps_$n.txt 2>&1 || exit $?
  SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstampsbb.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $n > $O/sstampsbb_$n.txt 2>&1 || exit $?
done
SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/nstamps_8192.txt 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 $O/timeline_8192.npz > $O/timeline_8192.txt 2>&1 || exit $?
echo R05F_DONE
