# round 4: 3-wave spill slots 80 -> 36 B/lane (row shuffles with a per-use lane id, branchless initial EPA facets, the stale cache entry invalidated by one dword)
# -- the whole GPU suite, then a same-box A/B against HEAD's build (_lib_var/tree: the tree scans)
export TMPDIR=/tmp
O=gpurun_out/r04m
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
V=gym-so100-c_amd/gym_so100/_lib_var; T=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_tree.so $T 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_tree.so $T 8192 3 > $O/ab8192.txt 2>&1 || exit $?
cat $O/ab8192.txt $O/ab65536.txt
echo R04M_DONE
