# broadphase restructure (sphere table + wave-wide OBB stage): GPU suite on the tree's build, A/B against the
# previous broadphase (ids2 build = HEAD 628444a), stage stamps of the new build
export TMPDIR=/tmp
O=gpurun_out/r03z
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_ids2.so $V/libso100_hip_bp2.so 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_ids2.so $V/libso100_hip_bp2.so 8192 3 > $O/ab8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps_bb.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 > $O/sstamps_8192.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_dstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton 8192 dyn > $O/dstamps_8192.txt 2>&1 || exit $?
echo R03Z_DONE
