# round 5: marginal cost of the box-box pairs (variant box2: their collider run twice per substep, the second result unused),
# interleaved with this tree's library at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05h
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for r in 1 2 3; do
  for n in 65536 8192; do
    timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/base_${n}_$r.json 2> $O/base_${n}_$r.err || exit $?
    SO100_LIB=$V/libso100_hip_box2.so timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/box2_${n}_$r.json 2> $O/box2_${n}_$r.err || exit $?
  done
done
echo R05H_DONE
