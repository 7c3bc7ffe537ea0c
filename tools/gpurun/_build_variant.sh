#!/bin/bash
# build a diagnostic/experimental variant of libso100_hip.so into gym_so100/_lib_var/<name>.so
# usage: tools/gpurun/_build_variant.sh <name> "<extra hipcc flags>"
set -e
NAME=$1; EXTRA=$2
W=/tmp/variant_$NAME
rm -rf $W && mkdir -p $W && cp -r /root/repo/gym-so100-c_amd /root/repo/include $W/
cd $W/gym-so100-c_amd/csrc && make clean >/dev/null && make -s HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize $EXTRA"
mkdir -p /root/repo/gym-so100-c_amd/gym_so100/_lib_var
cp ../gym_so100/_lib/libso100_hip.so /root/repo/gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_$NAME.so
echo built $NAME
