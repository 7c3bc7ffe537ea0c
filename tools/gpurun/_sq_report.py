"""Summary of the SQ counter passes of tools/gpurun/r06r.sh for one env count: each counter summed over the fused
step's launches and per launch, and the wave-cycle split (issue stalls vs issuing).
usage: python tools/gpurun/_sq_report.py <out dir> <n_envs>"""
import csv
import glob
import sys

d, n = sys.argv[1], sys.argv[2]
tot, launches = {}, {}
for f in glob.glob(f"{d}/sq*_{n}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "so100_fused_kernel" not in r["Kernel_Name"]:
            continue
        c = r["Counter_Name"]
        tot[c] = tot.get(c, 0.0) + float(r["Counter_Value"])
        launches.setdefault(c, set()).add(r["Dispatch_Id"])
print(f"# so100_fused_kernel at {n} envs: counters summed over the launches and per launch")
for c in sorted(tot):
    k = len(launches[c])
    print(f"{c:22s} total {tot[c]:.4g}  per launch {tot[c] / k:.4g}  ({k} launches)")
w = tot.get("SQ_WAVE_CYCLES")
if w:
    parts = {c: tot.get(c, 0.0) / w for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
    print("# SQ_WAVE_CYCLES = " + " + ".join(f"{c[3:]} {100 * v:.0f} %" for c, v in parts.items()))
