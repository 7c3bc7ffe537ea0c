# round 4 closing measurements on the final kernels: the GPU suite, a same-box A/B against the tree-scan build
# (_lib_var/tree: before the 3-wave spill cuts), the default bench line (65,536 envs + CPU baseline), the
# shard sizes (32,768 / 16,384 / 8,192 envs per GPU), PGS, rocprofv3 kernel stats, per-step PMC traffic at 65,536
# and 8,192 envs, the fused kernel's wave timeline at 8,192 envs (_lib_var/timeline), the GPU suite and smoke
export TMPDIR=/tmp
O=gpurun_out/r04n
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
V=gym-so100-c_amd/gym_so100/_lib_var; T=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_tree.so $T 65536 2 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_tree.so $T 8192 2 > $O/ab8192.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
for n in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --total-envs $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs.log 2>&1 || exit $?
for cfg in "fused 65536" "fused 8192"; do
  set -- $cfg
  B="python bench.py --total-envs $2 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  P=$O/pmc_$1_$2
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
  python tools/gpurun/pmc_step_traffic.py $P $2 $1 newton 40 5 $O/r04_pmc_step_$1_newton_$2.json > $P.traffic.log 2>&1 || exit $?
done
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_timeline.so timeout -k 10 200 python tools/gpurun/_fused_timeline.py 8192 $O/timeline_8192.npz > $O/timeline_8192.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo R04N_DONE
