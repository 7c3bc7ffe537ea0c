"""Diagnostic: per-phase cycle attribution of the step kernel (stamps build via SO100_LIB)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = SO100VecEnv(n, device="cuda:0", debug=True)
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for i in range(30):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
torch.cuda.synchronize()
acc = np.zeros(7)
ncon, iters = [], []
for i in range(5):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    d = env.debug.cpu().numpy()
    acc += d[::4, 88:95].mean(0)
    ncon.append(d[:, 0]); iters.append(d[:, 1])
acc /= 5
names = ["S1-S2 serial", "S3 collision", "S4-S7 setup", "PGS friction+limits", "PGS contacts", "S9 euler/debug", "final+epilogue"]
tot = acc.sum()
out = {k: float(v) for k, v in zip(names, acc)}
print(json.dumps(out, indent=1))
for k, v in zip(names, acc):
    print(f"{k:22s} {v/1e6:8.3f} Mcyc  {100*v/tot:5.1f}%")
nc = np.concatenate(ncon); it = np.concatenate(iters)
print("ncon last substep: mean %.2f, hist %s" % (nc.mean(), np.bincount(nc.astype(int), minlength=17)[:17].tolist()))
print("PGS iterations last substep: mean %.1f, frac==100 %.3f" % (it.mean(), (it == 100).mean()))
nm = nc.reshape(-1, 4).max(1)
print("wave-max ncon mean %.2f" % nm.mean())
