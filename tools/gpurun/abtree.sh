# same-box A/B of two whole trees (kernels + Python + bench.py), interleaved: tree A = abtree/<a> (an old revision
# built by _build_tree.sh), tree B = this tree.  usage: bash tools/gpurun/abtree.sh <out> <a> [envs] [reps] [steps]
export TMPDIR=/tmp
O=$1; A=$2; N=${3:-8192}; R=${4:-3}; S=${5:-200}
mkdir -p $O
for r in $(seq 1 $R); do
  (cd abtree/$A && timeout -k 10 200 python bench.py --total-envs $N --no-cpu-baseline --steps $S --contact-steps 0) > $O/ab_A_${N}_$r.json 2> $O/ab_A_${N}_$r.err || exit $?
  timeout -k 10 200 python bench.py --total-envs $N --no-cpu-baseline --steps $S --contact-steps 0 > $O/ab_B_${N}_$r.json 2> $O/ab_B_${N}_$r.err || exit $?
done
python - "$O" "$N" "$R" <<'PY'
import json, sys
o, n, r = sys.argv[1], sys.argv[2], int(sys.argv[3])
for v in "AB":
    vals = [json.load(open(f"{o}/ab_{v}_{n}_{i}.json"))["value"] / 1e6 for i in range(1, r + 1)]
    print(v, n, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / len(vals)))
PY
