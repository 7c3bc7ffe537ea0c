# round 4: the deep-fold / overflow parity tests (the ensemble gate with the FMA-contracted fp32 floor)
export TMPDIR=/tmp
O=gpurun_out/r04h
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rA --timeout 400 --timeout-method thread -s \
  -k "arm_contact or overflow or self_collision or base_contact or pad_link or cube_on_base" > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
echo R04H_DONE
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
