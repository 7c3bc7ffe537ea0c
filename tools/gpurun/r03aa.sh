# cube-table collapse without the 8-slot compaction (bb2 = the tree's build) vs HEAD 0dcdb1f (base3): GPU suite, A/B
export TMPDIR=/tmp
O=gpurun_out/r03aa
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_base3.so $V/libso100_hip_bb2.so 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_base3.so $V/libso100_hip_bb2.so 8192 3 > $O/ab8192.txt 2>&1 || exit $?
echo R03AA_DONE
