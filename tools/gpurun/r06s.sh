# round 6: the order kernel as one workgroup per XCD range: its GPU tests, its launch time (rocprofv3 stats at 65,536
# and 8,192 envs), and a same-box A/B against the one-workgroup order kernel (oldorder: HEAD before the change),
# interleaved, 3 runs each, 300 steps
export TMPDIR=/tmp
O=gpurun_out/r06s
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py -v --timeout 200 --timeout-method thread -rf > $O/pytest_order.log 2>&1; rc=$?
tail -3 $O/pytest_order.log
if [ $rc -ne 0 ]; then exit $rc; fi
for n in 65536 8192; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_$n -o tr --output-format csv -- python bench.py --total-envs $n --steps 60 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/tr_$n.log 2>&1 || exit $?
done
run() {  # tag, n, r
  L=""; [ $1 != cur ] && L=$V/libso100_hip_$1.so
  SO100_LIB=$L timeout -k 10 200 python bench.py --total-envs $2 --no-cpu-baseline --steps 300 --contact-steps 0 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err
}
for n in 65536 8192; do
  for r in 1 2 3; do
    for v in oldorder cur; do run $v $n $r || exit $?; done
  done
done
python - $O <<'PY'
import json, sys, csv, glob
o = sys.argv[1]
for n in (65536, 8192):
    for f in glob.glob(f"{o}/tr_{n}/*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if "order" in r["Name"] or "fused" in r["Name"]:
                print(n, r["Name"][:60], "avg us", round(float(r["AverageNs"]) / 1e3, 2))
    for v in ("oldorder", "cur"):
        vals = [json.loads(open(f"{o}/{v}_{n}_{r}.json").read().strip().splitlines()[-1])["value"] / 1e6 for r in (1, 2, 3)]
        print(n, v, " ".join(f"{x:.3f}" for x in vals), "mean %.3f" % (sum(vals) / 3))
PY
echo R06S_DONE
