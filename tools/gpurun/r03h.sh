# round-3 pass H: stage / Newton phase stamps at the 8-GPU shard (8,192 envs), EPA and MPR; the heavy PGS test
export TMPDIR=/tmp
O=gpurun_out/r03h
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for c in epa mpr; do
  CONVEX=$c SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/stage_8192_$c.txt 2>&1 || exit $?
done
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py 8192 > $O/newton_8192.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "heavy" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
echo R03H_DONE
