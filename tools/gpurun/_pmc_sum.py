"""Sum rocprofv3 --pmc counters over the so100 dispatches of a pass directory, per kernel and total
(diagnostics: tools/gpurun/_gpu_icache.sh).  usage: python tools/gpurun/_pmc_sum.py <dir> [<dir> ...]"""
import collections, csv, glob, sys

for d in sys.argv[1:]:
    tot = collections.defaultdict(float)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "so100" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("so100::", "").replace("void ", "")
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    print(d)
    for c in sorted(tot):
        print(f"  {c:32s} {tot[c]:.4g}")
    for k in sorted(per):
        print("   ", k, " ".join(f"{c}={v:.3g}" for c, v in sorted(per[k].items())))
