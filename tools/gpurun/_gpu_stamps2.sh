# stage stamps at N envs (split step): the full build vs the broadphase-only MPR build: gpurun_out/stamps2/*
export TMPDIR=/tmp
O=gpurun_out/stamps2
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
N=${1:-8192}
for v in sstamps sstampsbroad; do
  SO100_FUSED=0 SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $N > $O/${v}_$N.txt 2>&1 || exit $?
  echo "== $v"; cat $O/${v}_$N.txt
done
