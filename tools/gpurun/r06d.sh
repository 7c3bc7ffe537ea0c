# round 6 closing-style measurements on this tree: same-box A/B against round 5's closing tree (abtree/r05 = f9234e6) at
# 65,536 and 8,192 envs (VERDICT r5 item 1's rate cost), the driver's window on both, PMC traffic per step for the
# bench sizes and configs[3] / configs[4] (hash-tied: pmc_step_traffic.py reads each profiled run's own library hash),
# rocprofv3 kernel stats, then the bench lines that quote the PMC files.
export TMPDIR=/tmp
O=gpurun_out/r06d
rm -rf $O; mkdir -p $O
bash tools/gpurun/abtree.sh $O/ab65536 r05 65536 3 300 > $O/ab_65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05 8192 3 300 > $O/ab_8192.txt 2>&1 || exit $?
for r in 1 2 3; do
  (cd abtree/r05 && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) > $O/drv_r05_$r.json 2> $O/drv_r05_$r.err || exit $?
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_cur_$r.json 2> $O/drv_cur_$r.err || exit $?
done
pmc() {  # name, bench args, n
  P=$O/pmc_$1
  B="python bench.py $2 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || return $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || return $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || return $?
  python tools/gpurun/pmc_step_traffic.py $P $3 fused newton 40 5 $O/r06_pmc_step_$4.json > $P.traffic.log 2>&1 || return $?
}
pmc base65536 "--total-envs 65536" 65536 fused_newton_65536 || exit $?
pmc base8192 "--total-envs 8192" 8192 fused_newton_8192 || exit $?
pmc goal16384 "--total-envs 16384 --task so100_goal" 16384 goal_fused_newton_16384 || exit $?
pmc dr8192 "--total-envs 8192 --dr" 8192 dr_fused_newton_8192 || exit $?
cp $O/r06_pmc_step_*.json profiles/ || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace8192 -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace8192.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
timeout -k 10 300 python bench.py --total-envs 16384 --task so100_goal > $O/bench_goal_16384.json 2> $O/bench_goal_16384.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --dr > $O/bench_dr_8192.json 2> $O/bench_dr_8192.err || exit $?
echo R06D_DONE
