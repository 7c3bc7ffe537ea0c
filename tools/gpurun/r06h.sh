# round 6: the GPU suite on the current kernels (row EPA witness, the table snap's vertex by the hull support, the
# top-face rule by the hull support, the gradient-noise Newton stop, PGS kResident 6), then a same-box A/B at 8,192 and
# 65,536 envs: r05 (abtree/r05), prev (lib_var/base: the row witness, scanned snap / top-face vertex), cur (this tree)
export TMPDIR=/tmp
O=gpurun_out/r06h
rm -rf $O; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
V=gym-so100-c_amd/gym_so100/_lib_var
run() {  # tag, n, r
  if [ $1 = r05 ]; then
    (cd abtree/r05 && timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0) > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  elif [ $1 = prev ]; then
    SO100_LIB=$V/libso100_hip_base.so timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  else
    timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
  fi
}
for n in 8192 65536; do
  for r in 1 2 3; do
    for v in r05 prev cur; do run $v $n $r || exit $?; done
  done
done
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (8192, 65536):
    for v in ("r05", "prev", "cur"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
print("pgs", json.loads(open(f"{o}/bench_pgs.json").read().strip().splitlines()[-1])["value"] / 1e6)
PY
echo R06H_DONE
