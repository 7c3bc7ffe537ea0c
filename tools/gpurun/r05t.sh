# round 5: 65,536 and 32,768 envs, the 3-wave build (default above 2 waves per SIMD) against the 2-wave build forced
# (SO100_FUSED_WAVES=2: iterative-ILP scheduler, 256 VGPRs), same box, interleaved
export TMPDIR=/tmp
O=gpurun_out/r05t
rm -rf $O; mkdir -p $O
for r in 1 2; do
  for n in 65536 32768; do
    timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/w3_${n}_$r.json 2> $O/w3_${n}_$r.err || exit $?
    SO100_FUSED_WAVES=2 timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/w2_${n}_$r.json 2> $O/w2_${n}_$r.err || exit $?
  done
done
echo R05T_DONE
