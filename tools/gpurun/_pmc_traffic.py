"""Solver-kernel HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> JSON.

usage: python tools/gpurun/_pmc_traffic.py <pmc dir> <envs per solver launch> <out.json>
FETCH_SIZE/WRITE_SIZE are in KB (MI355X_MICROARCH.md, HBM/rocprofv3): memory-side L2->fabric bytes, one
counter per pass.  The last 20 solver dispatches of each pass are averaged.  gfx950 reports half the
bytes of 16-B/lane streaming reads in FETCH_SIZE; the solver's reads are 16-B/lane dwordx4, so the
fetch figure is doubled (the guide's correction) and both raw and corrected values are recorded.

VALU work ("report VALU-busy beside the HBM fraction"): SQ_INSTS_VALU (wave instructions
per dispatch) per kernel, and the VALU instructions of one env step of the whole batch
(10 solver + 11 stage launches per chunk, x chunks).  bench.py turns the latter into the VALU issue
share of the timed run: insts x 2 cycles (a wave64 VALU op holds a SIMD-32 for 2 cycles,
MI355X_MICROARCH.md) / (step time x 2.4 GHz x 1024 SIMDs).  Counter passes serialise dispatches, so a
per-dispatch busy figure from GRBM_GUI_ACTIVE would miss the chunks' overlap; it is recorded as
valu_issue_frac_serialised for reference only.

usage: python tools/gpurun/_pmc_traffic.py <pmc dir> <envs per solver launch> <out.json> [chunks] [solver]
solver: newton (so100_newton_kernel), pgs (so100_pgs_kernel; default for old profiles) or fused
(so100_fused_kernel: one launch per step, chunks = 1).  The Newton
kernel's reads mix 16-B J rows with 4-B header loads; the same x2 correction is applied (the J rows
dominate) and it is marked uncalibrated in the JSON.
"""
import csv, glob, json, sys

SOLVER = sys.argv[5] if len(sys.argv) > 5 else "pgs"
KERNEL = f"so100_{SOLVER}_kernel"      # solver "fused": so100_fused_kernel, the whole step in one launch


def per_launch(pattern, counter):
    vals = []
    for f in glob.glob(pattern):
        rows = [r for r in csv.DictReader(open(f)) if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        vals += [float(r["Counter_Value"]) for r in rows[-20:]]
    return sum(vals) / len(vals) if vals else None

d, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
insts = per_launch(d + "/sq*counter_collection.csv", "SQ_INSTS_VALU")
gui = per_launch(d + "/misc*counter_collection.csv", "GRBM_GUI_ACTIVE")
chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 1


def kernel_mean(pattern, counter, name):
    vals = []
    for f in glob.glob(pattern):
        rows = [r for r in csv.DictReader(open(f)) if name in r["Kernel_Name"] and r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        vals += [float(r["Counter_Value"]) for r in rows[-20:]]
    return sum(vals) / len(vals) if vals else 0.0


per_kernel = {k: kernel_mean(d + "/sq*counter_collection.csv", "SQ_INSTS_VALU", k)
              for k in (KERNEL, "so100_stage_kernel<0,", "so100_stage_kernel<1,", "so100_stage_kernel<2,")}
if SOLVER == "fused":
    step_insts = chunks * per_kernel[KERNEL]
else:
    step_insts = chunks * (10 * per_kernel[KERNEL] + per_kernel["so100_stage_kernel<0,"] +
                           9 * per_kernel["so100_stage_kernel<1,"] + per_kernel["so100_stage_kernel<2,"])
fetch = per_launch(d + "/fetch*counter_collection.csv", "FETCH_SIZE")
write = per_launch(d + "/write*counter_collection.csv", "WRITE_SIZE")
fx = 1 if SOLVER == "fused" else 2
res = {"kernel": KERNEL, "n_envs": n, "fetch_correction": "x2 (16-B/lane reads)" if SOLVER == "pgs" else
       ("none (4-B/lane state loads and scalar model loads; the x2 16-B/lane correction does not apply)"
        if SOLVER == "fused" else "x2 (J rows 16-B/lane; 4-B header loads uncalibrated)"),
       "fetch_kb_raw": fetch, "write_kb": write,
       "hbm_bytes_per_launch": (fx * fetch + write) * 1024 if fetch is not None and write is not None else None,
       "sq_insts_valu": insts, "grbm_gui_active": gui, "chunks": chunks,
       "valu_insts_per_kernel": per_kernel, "valu_insts_per_step": step_insts,
       "valu_issue_frac_serialised": (insts * 2.0) / (gui / 8.0 * 1024.0) if insts and gui else None,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), steady state (after 60 warmup steps), "
                 "mean of the last 20 dispatches of the kernel; FETCH doubled per the gfx950 16-B/lane correction "
                 "(not for the fused kernel)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
