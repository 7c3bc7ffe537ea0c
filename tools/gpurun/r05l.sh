# round 5: PGS at 65,536 envs — is the split path's per-env contact record stride (643 slots x 448 B = 288 KB per env)
# a cost? variant cap32 (the record cut to 32 slots, 14 KB per env; timing only: an env past 32 contacts would spill
# into its neighbour's record) against this tree, interleaved; and the env chunk count / step graphs; then the
# default bench line again, now that the closing PMC files (profiles/r05_pmc_step_*.json) match the library
export TMPDIR=/tmp
O=gpurun_out/r05l
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
P="python bench.py --solver pgs --no-cpu-baseline --steps 60 --contact-steps 0"
for r in 1 2; do
  timeout -k 10 200 $P > $O/base_$r.json 2> $O/base_$r.err || exit $?
  SO100_LIB=$V/libso100_hip_cap32.so timeout -k 10 200 $P > $O/cap32_$r.json 2> $O/cap32_$r.err || exit $?
done
for c in 2 3; do
  SO100_CHUNKS=$c timeout -k 10 200 $P > $O/chunks$c.json 2> $O/chunks$c.err || exit $?
done
SO100_GRAPH=1 timeout -k 10 200 $P > $O/graph.json 2> $O/graph.err || exit $?
SO100_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --contact-steps 0 > $O/split_base.json 2> $O/split_base.err || exit $?
SO100_FUSED=0 SO100_LIB=$V/libso100_hip_cap32.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --contact-steps 0 > $O/split_cap32.json 2> $O/split_cap32.err || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo R05L_DONE
