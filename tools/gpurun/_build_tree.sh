#!/bin/bash
# export git revision <rev> (the whole tree: kernels, Python, bench.py) to abtree/<name>/ and build its libraries
# here, so a GPU-box A/B can run the old revision's own bench.py beside HEAD's across ABI changes
# usage: tools/gpurun/_build_tree.sh <name> <rev>
set -e
NAME=$1; REV=$2
D=/root/repo/abtree/$NAME
rm -rf $D && mkdir -p $D
git -C /root/repo archive $REV | tar -x -C $D
make -s -j8 -C $D/gym-so100-c_amd/csrc
make -s -C $D/oracle
echo built $NAME from $REV in $D
