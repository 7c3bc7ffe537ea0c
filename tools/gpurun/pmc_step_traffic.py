"""HBM traffic and VALU work of ONE env step (every kernel of the step) from rocprofv3 --pmc passes -> JSON.

usage: python tools/gpurun/pmc_step_traffic.py <pmc dir> <n_envs> <mode> <solver> <warmup> <steps> <out.json>

The passes profile `bench.py --total-envs n --warmup W --steps S --contact-steps 0 --no-kernel-timing
--no-cpu-baseline` (fetch*: FETCH_SIZE, write*: WRITE_SIZE, sq*: SQ_INSTS_VALU; one counter block per pass,
MI355X_MICROARCH.md).  The step's kernels (stage / solver / fused / order) dispatch P times per step; the last
S x P dispatches (the timed steps) are summed and divided by S.  FETCH_SIZE and WRITE_SIZE are in KB
(memory-side L2 -> fabric requests).  gfx950 tallies a 16-B/lane streaming read at half its bytes in
FETCH_SIZE; the step's loads are mostly 4-B/lane and scalar, so hbm_bytes_per_step uses the raw count and
hbm_bytes_per_step_fetch_x2 is the upper bound with every read doubled.  bench.py reads the JSON
(profiles/r06_pmc_step_[goal_|dr_]<mode>_<solver>_<n>.json) for roofline.traffic, which it reports only when the
file's lib_source_hash equals the loaded library's.  That hash is the one the PROFILED processes loaded: each pass's
bench.py stdout (<pmc dir>.<pass>.log, the JSON line's roofline.lib_source_hash) is read, and the passes must agree
(round 6, ADVICE r5: a rebuild between profiling and this script no longer relabels the profile).
"""
import csv
import glob
import json
import os
import sys

STEP_KERNELS = ("so100_stage_kernel", "so100_newton_kernel", "so100_pgs_kernel", "so100_fused_kernel",
                "so100_order_kernel")


def step_rows(pattern, counter):
    rows = []
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in STEP_KERNELS):
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def per_step(rows, warmup, steps):
    total = warmup + steps
    if not rows or len(rows) % total:
        raise SystemExit(f"{len(rows)} step-kernel dispatches are not a multiple of {total} steps")
    p = len(rows) // total
    last = rows[-steps * p:]
    return sum(v for _, v, _ in last) / steps, p


def profiled_hashes(d):
    """roofline.lib_source_hash of every profiled bench.py run (<pmc dir>.<pass>.log: its one JSON line)"""
    out = []
    for f in sorted(glob.glob(d.rstrip("/") + ".*.log")):
        for line in open(f, errors="replace"):
            if line.startswith("{") and '"roofline"' in line:
                out.append(json.loads(line)["roofline"]["lib_source_hash"])
    if not out:
        raise SystemExit(f"no bench.py JSON line in {d}.*.log: the profiled runs' library hash is unknown")
    return out


def main():
    d, n, mode, solver, warmup, steps, out = sys.argv[1:8]
    n, warmup, steps = int(n), int(warmup), int(steps)
    fetch, p = per_step(step_rows(d + "/fetch*counter_collection.csv", "FETCH_SIZE"), warmup, steps)
    write, _ = per_step(step_rows(d + "/write*counter_collection.csv", "WRITE_SIZE"), warmup, steps)
    valu = None
    if glob.glob(d + "/sq*counter_collection.csv"):
        valu, _ = per_step(step_rows(d + "/sq*counter_collection.csv", "SQ_INSTS_VALU"), warmup, steps)
    hashes = profiled_hashes(d)
    if len(set(hashes)) != 1:
        raise SystemExit(f"the profiled passes' bench.py lines name {sorted(set(hashes))} library hashes")
    res = {"n_envs": n, "mode": mode, "solver": solver, "dispatches_per_step": p,
           "lib_source_hash": hashes[0], "hash_source": f"{len(hashes)} profiled bench.py lines ({d}.*.log)",
           "fetch_kb_per_step": fetch, "write_kb_per_step": write,
           "hbm_bytes_per_step": (fetch + write) * 1024, "hbm_bytes_per_step_fetch_x2": (2 * fetch + write) * 1024,
           "hbm_bytes_per_env_step": (fetch + write) * 1024 / n, "valu_insts_per_step": valu,
           "file": os.path.basename(out),
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU (separate passes) over bench.py "
                     f"--total-envs {n} --warmup {warmup} --steps {steps}: the last {steps} steps' {p} step-kernel "
                     f"dispatches each, summed per step"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
