# A/B on one box (gpurun_out/ab2/*): in-tree build vs library variants, bench at 65,536 and 8,192 envs,
# twice each, alternating.  usage: bash tools/gpurun/_gpu_ab2.sh variant1 [variant2 ...]
export TMPDIR=/tmp
O=gpurun_out/ab2
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for i in 1 2; do
  for n in ${NS:-65536 8192}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/base_${n}_$i.json 2>$O/err || exit $?
    for v in "$@"; do
      SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/${v}_${n}_$i.json 2>$O/err || exit $?
    done
  done
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f); done
echo AB2DONE
