# round 6: where does this round's rate go at 65,536 and 8,192 envs?  One box, interleaved, 3 runs each:
# r05 (abtree/r05 = f9234e6, its own bench.py), base (this tree's kernels, with the gradient-noise Newton stop),
# pool5 (base with round 5's pool size and relaxed take: -DSO100_POOL_R5), phys5 (base with round 5's EPA witness,
# Newton stop and no table-face snap: -DSO100_NO_FEAT -DSO100_NEWTON_RELSTOP -DSO100_NO_SNAP)
export TMPDIR=/tmp
O=gpurun_out/r06f
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 65536 8192; do
  for r in 1 2 3; do
    (cd abtree/r05 && timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0) > $O/r05_${n}_$r.json 2> $O/r05_${n}_$r.err || exit $?
    for v in base pool5 phys5; do
      SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/${v}_${n}_$r.json 2> $O/${v}_${n}_$r.err || exit $?
    done
  done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (65536, 8192):
    for v in ("r05", "base", "pool5", "phys5"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06F_DONE
