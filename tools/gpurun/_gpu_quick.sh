# quick GPU check: parity tests, bench line, per-kernel trace (writes gpurun_out/q/*)
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -rA -x > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
echo QDONE
