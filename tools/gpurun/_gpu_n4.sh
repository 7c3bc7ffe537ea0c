# split-path Newton kernel built for 4 waves per SIMD (128 VGPRs, 72 B/lane scratch) vs the product build (3): gpurun_out/n4/*
export TMPDIR=/tmp
O=gpurun_out/n4
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for i in 1 2; do for lib in product n4; do
  L=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so; [ $lib != product ] && L=$V/libso100_hip_$lib.so
  for n in 65536; do
    SO100_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/${lib}_${n}_$i.json 2>>$O/err || exit $?
  done
done; done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f); done
