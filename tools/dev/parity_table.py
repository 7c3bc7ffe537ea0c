"""Markdown table of the GPU parity summaries in a `pytest -m gpu -s` log (TF.summary lines): per class and solver,
the GPU's qvel rel. error median / p90 / max against the fp64 oracle, the fp32 restatement's and the 1-ulp perturbed
fp64's on the same states, and the share within north_star's 1e-4.
usage: python tools/dev/parity_table.py <pytest log>"""
import re
import sys

pat = re.compile(r"\[(?:ee )?(newton|pgs)?\s*([^\]]*?)\] (\d+) env-steps[^|]*\| median / p90 / max: qvel rel GPU "
                 r"([0-9e.+-]+) / ([0-9e.+-]+) / ([0-9e.+-]+) \(fp32 oracle ([0-9e.+-]+) / ([0-9e.+-]+) / ([0-9e.+-]+); "
                 r"fp64 under a 1-ulp input perturbation ([0-9e.+-]+) / ([0-9e.+-]+) / ([0-9e.+-]+)\), within 1e-4: ([0-9.]+)")
ee = re.compile(r"\[ee (newton|pgs)\]")
print("| class | solver | env steps | GPU qvel rel. median / p90 / max | fp32 restatement | fp64, 1-ulp perturbed | GPU within 1e-4 |")
print("|---|---|---|---|---|---|---|")
seen = set()
for line in open(sys.argv[1], errors="replace"):
    for m in pat.finditer(line):
        g = m.groups()
        solver, cls = g[0], g[1].strip()
        e = ee.search(m.group(0))
        if e:
            solver, cls = e.group(1), "EE / mocap weld"
        if not solver:                       # "[newton random actions]" style: solver first word of the label
            parts = cls.split(" ", 1)
            solver, cls = parts[0], parts[1] if len(parts) > 1 else ""
        key = (cls, solver)
        if key in seen:
            continue
        seen.add(key)
        print(f"| {cls} | {solver} | {g[2]} | {g[3]} / {g[4]} / {g[5]} | {g[6]} / {g[7]} / {g[8]} | "
              f"{g[9]} / {g[10]} / {g[11]} | {float(g[12]):.3f} |")
