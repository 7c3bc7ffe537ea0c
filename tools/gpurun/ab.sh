# A/B of two library builds on one box, interleaved: bash tools/gpurun/ab.sh <out> <libA> <libB> [envs] [reps]
export TMPDIR=/tmp
O=$1; A=$2; B=$3; N=${4:-8192}; R=${5:-3}
mkdir -p $O
for r in $(seq 1 $R); do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    SO100_LIB=$L timeout -k 10 200 python bench.py --total-envs $N --no-cpu-baseline --steps 200 --contact-steps 0 > $O/ab_${v}_${N}_$r.json 2> $O/ab_${v}_${N}_$r.err || exit $?
  done
done
python - "$O" "$N" "$R" <<'PY'
import json, sys
o, n, r = sys.argv[1], sys.argv[2], int(sys.argv[3])
for v in "AB":
    vals = [json.load(open(f"{o}/ab_{v}_{n}_{i}.json"))["value"] / 1e6 for i in range(1, r + 1)]
    print(v, n, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / len(vals)))
PY
