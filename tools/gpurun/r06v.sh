# round 6: the 2-wave build (8,192 envs) with and without the skipped cost after a quadratic-exact stop (f2skip:
# -DSO100_FUSED2_COSTSKIP), against prevcost (before the skip); same box, interleaved, 3 runs each, 300 steps
export TMPDIR=/tmp
O=gpurun_out/r06v
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
run() {  # tag, n, r
  L=""; [ $1 != cur ] && L=$V/libso100_hip_$1.so
  SO100_LIB=$L timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
}
for n in 8192; do
  for r in 1 2 3; do
    for v in prevcost cur f2skip; do run $v $n $r || exit $?; done
  done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (8192,):
    for v in ("prevcost", "cur", "f2skip"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06U_DONE
