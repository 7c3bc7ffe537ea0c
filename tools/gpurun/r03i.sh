# round-3 pass I: lane-parallel EPA horizon / facets -- EPA-class parity, product builds, 8,192 rate, stage stamps
export TMPDIR=/tmp
O=gpurun_out/r03i
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mpr_contact or self_collision or base or pad_link or arm_contact or product_builds or teacher_forced or heavy" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
CONVEX=epa SO100_FUSED=0 SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_sstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/stage_8192_epa.txt 2>&1 || exit $?
echo R03I_DONE
