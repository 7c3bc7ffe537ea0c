"""Spill / reload sites of a fused kernel in a device asm dump (make -C gym-so100-c_amd/csrc ru3 -> /tmp/so100_f3.s).
usage: python tools/dev/spill_sites.py [asm] [kernel-substring]
Prints each scratch access with its source line (the last non-zero .loc), its basic block's loop depth, and a summary
of the spill slots: which offsets are stored / reloaded where."""
import re, sys
from collections import defaultdict
path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/so100_f3.s"
kern = sys.argv[2] if len(sys.argv) > 2 else "so100_fused_kernelILb0ELi3E"
s = open(path).read().split("\n")
files = {}
for l in s:
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
    if m: files[m.group(1)] = m.group(2).split("/")[-1]
start = [i for i, l in enumerate(s) if re.match(r"_Z\S*" + kern + r"\S*:", l)][0]
end = [i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end")][0]
loc, depth = None, 0
slots = defaultdict(lambda: {"st": [], "ld": []})
for i in range(start, end):
    l = s[i]
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m and int(m.group(2)): loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
    m = re.search(r"Depth=(\d+)", l)
    if re.match(r"^\.LBB|^; %bb", l): depth = int(m.group(1)) if m else 0
    if "scratch_" in l:
        off = re.search(r"offset:(\d+)", l)
        off = int(off.group(1)) if off else 0
        kind = "st" if "store" in l else "ld"
        slots[off][kind].append((loc, depth))
        print(f"{i - start:7d} d{depth} {loc:24s} {l.strip()[:80]}")
print("\nslot  stores (line, loop depth)  |  reloads")
for off in sorted(slots):
    f = lambda v: ", ".join(f"{a}/d{d}" for a, d in v)
    print(f"{off:4d}  {f(slots[off]['st'])}  |  {f(slots[off]['ld'])}")
