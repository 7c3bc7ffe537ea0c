# round-3 pass G: heavy PGS outlier walk, EPA-class parity tests and the 8,192 rate after the EPA vertex cache
export TMPDIR=/tmp
O=gpurun_out/r03g
rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/dev/tf_outlier.py heavy pgs epa $O/heavy.npz > $O/outlier_heavy_pgs.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mpr_contact or heavy or teacher_forced or self_collision or base_contact or pad_link" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
echo R03G_DONE
