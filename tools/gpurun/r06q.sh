# round 6: the GPU suite (-s: every parity test's summary line, for tools/dev/parity_table.py) and smoke() on this tree
export TMPDIR=/tmp
O=gpurun_out/r06q
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc $?" >> $O/smoke.log
tail -2 $O/smoke.log
python tools/dev/parity_table.py $O/pytest_gpu.log > $O/parity_table.md
echo R06Q_DONE
