# round-3 final check on HEAD: GPU suite, smoke, the default bench line (65,536 envs + CPU baseline), the 8-GPU shard
# size, rocprofv3 kernel stats at 8,192 envs (the 2-wave build with the broadcast dynamics)
export TMPDIR=/tmp
O=gpurun_out/r03final
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_fused -o fused8192 --output-format csv -- python bench.py --total-envs 8192 --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_fused.log 2>&1 || exit $?
echo R03FINAL_DONE
