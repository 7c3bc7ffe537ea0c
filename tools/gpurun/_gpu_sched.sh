# scheduler-option variants of libso100_hip.so vs the product build: fused step at 8,192 envs and the
# default (split) step at 65,536, interleaved twice (gpurun_out/sched/*)
export TMPDIR=/tmp
O=gpurun_out/sched
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for i in 1 2; do for lib in product ilp trk bias0; do
  L=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so; [ $lib != product ] && L=$V/libso100_hip_$lib.so
  for n in 8192 65536; do
    SO100_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/${lib}_${n}_$i.json 2>>$O/err || exit $?
  done
done; done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f); done
