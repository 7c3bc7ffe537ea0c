# round 6: the GPU suite on the round's kernels (feature-witness EPA, table-face snap, hull-relative lowest vertex,
# Newton decrement stop, resident-sized pool), then the bench at 65,536 and 8,192 envs.  Test failures (rc 1) do not
# stop the script; a fault, abort or time limit does.
export TMPDIR=/tmp
O=gpurun_out/r06c
rm -rf $O; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_65536.json 2> $O/bench_65536.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --total-envs 8192 > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
echo R06C_DONE
