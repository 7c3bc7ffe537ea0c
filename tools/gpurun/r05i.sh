# round 5: same-box A/B of the box-box loops stopping at the wave's last polygon slot (this tree) against HEAD 4372fd4
# (abtree/r05x), 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05i
rm -rf $O; mkdir -p $O
bash tools/gpurun/abtree.sh $O/ab65536 r05x 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/abtree.sh $O/ab8192 r05x 8192 3 300 > $O/ab8192.txt 2>&1 || exit $?
echo R05I_DONE
