"""Summarise rocprofv3 SQ counter CSVs per step-pipeline kernel (last 4 dispatches of each)."""
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "so100" not in k:
            continue
        name = k.split("(")[0].replace("so100::", "").replace("void ", "")
        per[name][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    print(f.split("/")[-1])
    for name, d in per.items():
        ds = [d[k] for k in sorted(d)][-4:]
        avg = {c: sum(x.get(c, 0) for x in ds) / len(ds) for c in ds[0]}
        w = avg.get("SQ_WAVES", 1) or 1
        wc = avg.get("SQ_WAVE_CYCLES", 0)
        line = " ".join(f"{c.replace('SQ_', '')}={v / w:.0f}" for c, v in avg.items() if c != "SQ_WAVES")
        if wc:
            line += f" | active {avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait {avg.get('SQ_WAIT_ANY', 0) / wc:.2f}"
        print(f"  {name:28s} waves={w:.0f} {line}")
