# per-phase cycle attribution (stamps builds, split step) at the given shard size: gpurun_out/stamps/*
export TMPDIR=/tmp
O=gpurun_out/stamps
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
N=${1:-8192}
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $N > $O/stage_$N.txt 2>&1 || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_nstamps.so timeout -k 10 200 python tools/gpurun/_newton_stamps_report.py $N > $O/newton_$N.txt 2>&1 || exit $?
cat $O/stage_$N.txt $O/newton_$N.txt
