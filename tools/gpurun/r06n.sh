# round 6: Newton steps per solve on the GPU (debug build, last substep) with and without the quadratic-exact stop
export TMPDIR=/tmp
O=gpurun_out/r06n
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 8192 65536; do
  timeout -k 10 200 python tools/dev/newton_iters_gpu.py $n 60 >> $O/iters.txt 2>&1 || exit $?
  SO100_LIB=$V/libso100_hip_noquad.so timeout -k 10 200 python tools/dev/newton_iters_gpu.py $n 60 >> $O/iters.txt 2>&1 || exit $?
done
cat $O/iters.txt
