# A/B of library variants (gym_so100/_lib_var/libso100_hip_<name>.so) against the in-tree build on ONE box:
# bench (default steps) twice each, then a kernel trace of each in the bench's steady state.
# usage: bash tools/gpurun/_gpu_ab.sh name1 name2 ...   (writes gpurun_out/ab/*)
export TMPDIR=/tmp
O=gpurun_out/ab
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/base_$i.log 2>&1 || exit $?
  for n in "$@"; do
    SO100_LIB=$V/libso100_hip_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/${n}_$i.log 2>&1 || exit $?
  done
done
T="python bench.py --steps 20 --warmup 60 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o base --output-format csv -- $T > $O/trace_base.log 2>&1 || exit $?
for n in "$@"; do
  SO100_LIB=$V/libso100_hip_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o $n --output-format csv -- $T > $O/trace_$n.log 2>&1 || exit $?
done
for f in $O/*_[12].log; do echo $f $(grep -o '"value": [0-9.]*' $f); done
echo ABDONE
