"""Convex-collider phase cycles on the GPU (dev probe; needs the -DSO100_EPA_STAMPS library variant):
    SO100_LIB=.../libso100_hip_epastamps.so python tools/dev/epa_stamps.py [n] [fused]
Steps n bench envs 60 steps, then sums over 5 steps per row-item: GJK and EPA cycles, EPA iterations, and
inside EPA the nearest-facet scan, the support and the horizon + new facets."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
from gym_so100 import SO100VecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
lib = ctypes.CDLL(os.environ["SO100_LIB"])
env = SO100VecEnv(n, device="cuda:0", seed=0)
env.fused = len(sys.argv) > 2 and sys.argv[2] == "fused"
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for i in range(60):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 12)()
lib.so100_dev_epa_cycles(buf, 1)
for i in range(5):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
torch.cuda.synchronize()
lib.so100_dev_epa_cycles(buf, 0)
gjk, epa, items, eitems, eit, sup, hor, scan, h_vis, h_mask, h_fac, _ = list(buf)
print(f"{n} envs x 5 steps ({'fused' if env.fused else 'split'}): {items} row-items, {eitems} to EPA, {eit} EPA iterations "
      f"({eit / max(eitems, 1):.1f} per EPA item)")
print(f"  GJK {gjk / max(items, 1):.0f} cyc per item; EPA {epa / max(eitems, 1):.0f} cyc per EPA item")
print(f"  per EPA iteration: nearest-facet scan {scan / max(eit, 1):.0f}, support {sup / max(eit, 1):.0f}, "
      f"horizon + new facets {hor / max(eit, 1):.0f} cyc (visibility {(hor - h_vis - h_mask - h_fac) / max(eit, 1):.0f}, "
      f"twin test + horizon masks {h_vis / max(eit, 1):.0f}, bookkeeping {h_mask / max(eit, 1):.0f}, "
      f"new facets {h_fac / max(eit, 1):.0f})")
