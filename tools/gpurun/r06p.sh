# round 6: the quadratic-exact stop with the zones taken from the rows' own evaluations (the iterate's and the line
# search's first): cur against noquad (-DSO100_NO_QUADSTOP) at 8,192 and 65,536 envs, same box, interleaved, 3 runs
export TMPDIR=/tmp
O=gpurun_out/r06p
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
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
    for v in cur noquad; do run $v $n $r || exit $?; done
  done
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (8192, 65536):
    for v in ("cur", "noquad"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06J_DONE
