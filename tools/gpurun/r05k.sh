# round 5: same-box A/B of the box-box loops stopping at the wave's last polygon slot, sphere test unchanged (this tree) against HEAD 1c499a7
# (abtree/r05y), 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05k
rm -rf $O; mkdir -p $O
bash tools/gpurun/abtree.sh $O/ab65536 r05y 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05y 8192 3 300 > $O/ab8192.txt 2>&1 || exit $?
echo R05K_DONE
