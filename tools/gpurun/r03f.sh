# round-3 pass F: PGS with MuJoCo's QCQP iteration (deviation 6 removed): PGS parity tests, the outlier walk, PGS bench
export TMPDIR=/tmp
O=gpurun_out/r03f
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pgs or full_size" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_pgs.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_pgs.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/dev/tf_outlier.py mpr pgs epa $O/mpr_pgs_epa.npz > $O/outlier_mpr_pgs_epa.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --solver pgs > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
echo R03F_DONE
