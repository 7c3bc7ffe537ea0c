# collision-parity tests (no -x) and a bench A/B against the no-pads variant (writes gpurun_out/base/*)
export TMPDIR=/tmp
O=gpurun_out/base
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rA -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --solver pgs > $O/bench_pgs.json 2>$O/bench_pgs.err || exit $?
echo BDONE
