# round 4: first run of the uncapped contact list (ABI 14): GPU suite, smoke, bench lines at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r04a
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline --steps 200 > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
echo R04A_DONE
