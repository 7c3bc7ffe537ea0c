# round 5: the broadphase's sphere-test index pairs from one packed 16-B load per lane (this tree) against HEAD 69f68a6
# (abtree/r05w): bitwise checks (product builds, fused vs split), then a same-box A/B at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05n
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "product_builds or fused_step_matches_split" > $O/pytest.log 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab65536 r05w 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05w 8192 3 300 > $O/ab8192.txt 2>&1 || exit $?
echo R05N_DONE
