# round-3 pass K: one-load hull support (cell blocks), one division per EPA facet: parity subset, 8,192 rate, EPA stamps
export TMPDIR=/tmp
O=gpurun_out/r03k
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mpr_contact or self_collision or base or pad_link or arm_contact or product_builds or teacher_forced or heavy or hull_table or pad_contact" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_epastamps.so timeout -k 10 200 python tools/dev/epa_stamps.py 8192 fused > $O/epa_fused.txt 2>&1 || exit $?
echo R03K_DONE
