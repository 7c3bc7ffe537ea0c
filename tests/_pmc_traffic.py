"""Solver-kernel HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> JSON.

usage: python tests/_pmc_traffic.py <pmc dir> <n_envs> <out.json>
FETCH_SIZE/WRITE_SIZE are in KB (MI355X_MICROARCH.md, HBM/rocprofv3): memory-side L2->fabric bytes, one
counter per pass.  The last 20 solver dispatches of each pass are averaged.  gfx950 reports half the
bytes of 16-B/lane streaming reads in FETCH_SIZE; the solver's reads are 16-B/lane dwordx4, so the
fetch figure is doubled (the guide's correction) and both raw and corrected values are recorded.
"""
import csv, glob, json, sys

def per_launch(pattern, counter):
    vals = []
    for f in glob.glob(pattern):
        rows = [r for r in csv.DictReader(open(f)) if "pgs_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        vals += [float(r["Counter_Value"]) for r in rows[-20:]]
    return sum(vals) / len(vals) if vals else None

d, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
fetch = per_launch(d + "/fetch*counter_collection.csv", "FETCH_SIZE")
write = per_launch(d + "/write*counter_collection.csv", "WRITE_SIZE")
res = {"kernel": "so100_pgs_kernel", "n_envs": n,
       "fetch_kb_raw": fetch, "write_kb": write,
       "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), steady state (after 60 warmup steps), "
                 "mean of the last 20 solver dispatches; FETCH doubled per the gfx950 16-B/lane correction"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
