#!/bin/bash
# build libso100_hip.so of git revision <rev> into gym_so100/_lib_var/libso100_hip_<name>.so (A/B baselines)
# usage: tools/gpurun/_build_rev.sh <name> <rev>
set -e
NAME=$1; REV=$2
W=/tmp/rev_$NAME
rm -rf $W && mkdir -p $W
git -C /root/repo archive $REV gym-so100-c_amd/csrc include | tar -x -C $W
mkdir -p $W/gym-so100-c_amd/gym_so100/_lib
make -s -C $W/gym-so100-c_amd/csrc
mkdir -p /root/repo/gym-so100-c_amd/gym_so100/_lib_var
cp $W/gym-so100-c_amd/gym_so100/_lib/libso100_hip.so /root/repo/gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_$NAME.so
echo built $NAME from $REV
