# round 6 closing measurements, part 1 (the final kernels): per-step PMC traffic for the bench sizes and configs[3] /
# configs[4] and PGS at 65,536 (each file carries the profiled runs' own library hash), rocprofv3 kernel stats (65,536 / 8,192 / PGS),
# the fused kernel's wave timeline and the Newton stamps at 8,192 envs (variants of the same sources), smoke.
# Part 2 (r06z.sh) runs the bench lines, which quote the PMC files once they are in profiles/.
export TMPDIR=/tmp
O=gpurun_out/r06y
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
pmc() {  # name, bench args, n, out tag, mode, solver
  P=$O/pmc_$1
  B="python bench.py $2 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || return $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || return $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || return $?
  python tools/gpurun/pmc_step_traffic.py $P $3 $5 $6 40 5 $O/r06_pmc_step_$4.json > $P.traffic.log 2>&1 || return $?
}
pmc base65536 "--total-envs 65536" 65536 fused_newton_65536 fused newton || exit $?
pmc base32768 "--total-envs 32768" 32768 fused_newton_32768 fused newton || exit $?
pmc base16384 "--total-envs 16384" 16384 fused_newton_16384 fused newton || exit $?
pmc base8192 "--total-envs 8192" 8192 fused_newton_8192 fused newton || exit $?
pmc goal16384 "--total-envs 16384 --task so100_goal" 16384 goal_fused_newton_16384 fused newton || exit $?
pmc dr8192 "--total-envs 8192 --dr" 8192 dr_fused_newton_8192 fused newton || exit $?
pmc pgs65536 "--total-envs 65536 --solver pgs" 65536 split_pgs_65536 split pgs || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace8192 -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace8192.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs.log 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 $O/timeline_8192.npz > $O/timeline_8192.txt 2>&1 || exit $?
SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/nstamps_8192.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo R06Y_DONE
