# last check of the tree's build: GPU suite and smoke
export TMPDIR=/tmp
O=gpurun_out/r03last
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
echo R03LAST_DONE
