# round 5: the PGS kernel at a 2-wave register budget (176 VGPRs, no scratch) under the default, max-ilp, iterative-ilp
# and max-memory-clause schedulers, 65,536 envs, interleaved with this tree
export TMPDIR=/tmp
O=gpurun_out/r05s
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
P="python bench.py --solver pgs --no-cpu-baseline --steps 60 --contact-steps 0"
for r in 1 2; do
  timeout -k 10 200 $P > $O/base_$r.json 2> $O/base_$r.err || exit $?
  for v in pgsw2_default pgsw2_max-ilp pgsw2_iterative-ilp pgsw2_max-memory-clause; do
    SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 $P > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
  done
done
echo R05S_DONE
