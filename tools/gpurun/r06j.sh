# round 6: the quadratic-exact Newton stop: the GPU suite on this tree, then a same-box A/B, interleaved, 3 runs each,
# 300 steps: r05 (abtree/r05), cur (this tree), noquad (this tree with -DSO100_NO_QUADSTOP), at 8,192 and 65,536 envs
export TMPDIR=/tmp
O=gpurun_out/r06j
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
run() {  # tag, n, r
  if [ $1 = r05 ]; then
    (cd abtree/r05 && timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0) > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  else
    L=""; [ $1 = noquad ] && L=$V/libso100_hip_noquad.so
    SO100_LIB=$L timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  fi
}
for n in 8192 65536; do
  for r in 1 2 3; do
    for v in r05 cur noquad; do run $v $n $r || exit $?; done
  done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (8192, 65536):
    for v in ("r05", "cur", "noquad"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06J_DONE
