# Newton solver: GPU parity tests, then the bench line with each solver (writes gpurun_out/nw/*)
export TMPDIR=/tmp
O=gpurun_out/nw
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --solver newton > $O/bench_newton.json 2>$O/bench_newton.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_pgs.json 2>$O/bench_pgs.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o newton --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline --solver newton > $O/trace.log 2>&1 || exit $?
echo NWDONE
