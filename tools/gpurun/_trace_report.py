"""Per-kernel time per chunk-step from rocprofv3 kernel traces (the last N final-stage launches of each
trace; with C concurrent env chunks a step holds C chunk-steps, so wall is the step time / C).  A fused step
(so100_fused_kernel) is one launch: it marks the step itself."""
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*_kernel_trace.csv")):
    rows = [r for r in csv.DictReader(open(f)) if "so100" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    END = ("stage_kernel<2", "fused_kernel")
    finals = [i for i, r in enumerate(rows) if any(k in r["Kernel_Name"] for k in END)]
    if len(finals) < 3:
        continue
    a, b = finals[-11] if len(finals) > 11 else finals[0], finals[-1]
    tot = collections.Counter()
    for r in rows[a + 1:b + 1]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("so100::", "")
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    nsteps = sum(1 for r in rows[a + 1:b + 1] if any(k in r["Kernel_Name"] for k in END))
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6 / nsteps
    print(f.split("/")[-1].replace("_kernel_trace.csv", ""), f"wall {wall:.2f} ms per chunk-step, kernel ms per chunk-step:",
          ", ".join(f"{k} {v / nsteps:.2f}" for k, v in tot.most_common()))
