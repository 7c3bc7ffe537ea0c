# round 5: where the stage time goes on the current kernels: stage stamps (split path) with and without the box-box
# pairs split out (SO100_STAMP_BOXBOX: slot 0) at 65,536 and 8,192 envs; Newton stamps and the fused wave timeline
# at 8,192 envs; a same-box A/B of the per-XCD heavy-first order (this tree) against the global one (abtree/r05pre)
# at 65,536 and 8,192 envs, and this tree's per-step PMC traffic at 65,536
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
bash tools/gpurun/abtree.sh $O/ab65536 r05pre 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05pre 8192 3 300 > $O/ab8192.txt 2>&1 || exit $?
n=65536
B="python bench.py --total-envs $n --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
P=$O/pmc_fused_$n
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
python tools/gpurun/pmc_step_traffic.py $P $n fused newton 40 5 $O/r05_pmc_step_fused_newton_$n.json > $P.traffic.log 2>&1 || exit $?
echo R05F_DONE
