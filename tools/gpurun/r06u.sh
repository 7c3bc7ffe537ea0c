# round 6: no cost evaluation after a quadratic-exact stop (the product builds; the iterate is unchanged): the bitwise
# tests (product builds vs the debug build and the split path, the order test), then a same-box A/B against HEAD
# before the change (prevcost), interleaved, 3 runs each, 300 steps, 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r06u
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rf -k "order or pool_contention or newton_solver_parity or fused" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, n, r
  L=""; [ $1 != cur ] && L=$V/libso100_hip_$1.so
  SO100_LIB=$L timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
}
for n in 65536 8192; do
  for r in 1 2 3; do
    for v in prevcost cur; do run $v $n $r || exit $?; done
  done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (65536, 8192):
    for v in ("prevcost", "cur"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06U_DONE
