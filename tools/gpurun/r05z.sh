# round 5 closing measurements on the final kernels, part 1: the GPU suite, the shard sizes (32,768 / 16,384 / 8,192
# envs per GPU), PGS, rocprofv3 kernel stats (part 2, r05z2.sh: PMC traffic, then the default bench line quoting it)
export TMPDIR=/tmp
O=gpurun_out/r05z
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for n in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --total-envs $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs.log 2>&1 || exit $?
echo R05Z_DONE
