# round 5: the LLVM AMDGPU scheduling strategy for the fused step at 8,192 envs (the 2-wave build: no scratch under
# either strategy; the 3-wave build spills under both, so 65,536 is not a candidate), interleaved with this tree
export TMPDIR=/tmp
O=gpurun_out/r05p
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/base_$r.json 2> $O/base_$r.err || exit $?
  for st in max-ilp iterative-ilp; do
    SO100_LIB=$V/libso100_hip_sched_$st.so timeout -k 10 200 python bench.py --total-envs 8192 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/${st}_$r.json 2> $O/${st}_$r.err || exit $?
  done
done
echo R05P_DONE
