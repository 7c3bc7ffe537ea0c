# round-2 first GPU check (writes gpurun_out/r02a/*): parity tests, bench line, kernel traces at the
# 8-GPU shard size (8,192 envs) and the 1-GPU size, for the launch-gap / tail analysis.
export TMPDIR=/tmp
O=gpurun_out/r02a
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit $?
for n in 8192 65536; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$n -o t --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --total-envs $n > $O/trace_$n.log 2>&1 || exit $?
done
echo R02ADONE
