export TMPDIR=/tmp
O=gpurun_out/r01b
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo BDONE
