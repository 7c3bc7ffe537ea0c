# round 6: the 8,192-env shard (the 8-GPU point) after the row witness: one box, interleaved, 3 runs each, 300 steps:
# r05 (abtree/r05), base (this tree), lane0 (EPA's contact rebuilt on the staging lane), nofeat / nosnap / relstop
# (base with one of the round's changes switched off), phys5 (all three off); then 65,536 for r05 / base
export TMPDIR=/tmp
O=gpurun_out/r06g
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
run() {  # tag, n, r
  if [ $1 = r05 ]; then
    (cd abtree/r05 && timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0) > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  else
    SO100_LIB=$V/libso100_hip_$1.so timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  fi
}
for r in 1 2 3; do
  for v in r05 base lane0 nofeat nosnap relstop phys5; do run $v 8192 $r || exit $?; done
done
for r in 1 2 3; do
  for v in r05 base; do run $v 65536 $r || exit $?; done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n, vs in ((8192, ("r05", "base", "lane0", "nofeat", "nosnap", "relstop", "phys5")), (65536, ("r05", "base"))):
    for v in vs:
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06G_DONE
