# round 4: the fused 2- vs 3-wave build at 65,536 and 16,384 envs (same library, interleaved)
export TMPDIR=/tmp
O=gpurun_out/r04k
rm -rf $O; mkdir -p $O
for n in 65536 16384; do
  for r in 1 2 3; do
    for w in 2 3; do
      timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 --fused-build $w > $O/b_${n}_w${w}_$r.json 2> $O/b_${n}_w${w}_$r.err || exit $?
    done
  done
done
python - $O <<'PY'
import json, sys, glob
o = sys.argv[1]
for n in (65536, 16384):
    for w in (2, 3):
        v = [json.load(open(f))["value"] / 1e6 for f in sorted(glob.glob(f"{o}/b_{n}_w{w}_*.json"))]
        print(n, "waves", w, " ".join(f"{x:.3f}" for x in v), "mean %.3f" % (sum(v) / len(v)))
PY
echo R04K_DONE
