# round 5 closing measurements, part 2 (same tree as r05z.sh): per-step PMC traffic at 65,536 / 16,384 / 8,192 envs
# (files carry the library's source hash; copied into this box's profiles/ so that the default bench line, run next
# with its CPU baseline, quotes them), the fused kernel's wave timeline and the stage / Newton stamps at 8,192 envs
# (variants built from the same sources), smoke
export TMPDIR=/tmp
O=gpurun_out/r05z2
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 65536 16384 8192; do
  B="python bench.py --total-envs $n --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  P=$O/pmc_fused_$n
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
  python tools/gpurun/pmc_step_traffic.py $P $n fused newton 40 5 $O/r05_pmc_step_fused_newton_$n.json > $P.traffic.log 2>&1 || exit $?
done
cp $O/r05_pmc_step_fused_newton_*.json profiles/ || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 $O/timeline_8192.npz > $O/timeline_8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/sstamps_8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstampsbb.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/sstampsbb_8192.txt 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/nstamps_8192.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for r in 1 2; do   # the 16,384-env shard: the 3-wave build (default) against the 2-wave build forced (iterative-ILP scheduler)
  timeout -k 10 200 python bench.py --total-envs 16384 --no-cpu-baseline --steps 200 --contact-steps 0 > $O/w3_16384_$r.json 2> $O/w3_16384_$r.err || exit $?
  SO100_FUSED_WAVES=2 timeout -k 10 200 python bench.py --total-envs 16384 --no-cpu-baseline --steps 200 --contact-steps 0 > $O/w2_16384_$r.json 2> $O/w2_16384_$r.err || exit $?
done
echo R05Z2_DONE
