"""Diagnostic: per-phase cycles of the Newton solver kernel (last substep of a step); SO100_STAMPS build via
SO100_LIB.  usage: SO100_LIB=<stamps build> python tools/gpurun/_newton_stamps_report.py [n]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = SO100VecEnv(n, device="cuda:0", debug=True, solver="newton")
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for i in range(60):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
acc, it = np.zeros(8), 0.0
rows = []
for i in range(3):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    d = env.debug.cpu().numpy()
    acc += d[::4, 88:96].mean(0)
    rows.append(d[::4, 88:96])
    it += d[:, 1].mean()
acc /= 3
names = ["load record", "warmstart choice", "rows + gradient", "Hessian", "Cholesky + solves", "line search",
         "move + cost", "tail (wait for the wave)"]
print(f"Newton steps per substep (env mean) {it / 3:.2f}")
for k, v in zip(names, acc):
    print(f"{k:26s} {v / 1e3:8.1f} Kcyc  {100 * v / acc.sum():5.1f}%")
R = np.concatenate(rows)
top = R[np.argsort(R.sum(1))[-max(1, len(R) // 100):]].mean(0)
print("slowest 1% of waves:")
for k, v in zip(names, top):
    print(f"{k:26s} {v / 1e3:8.1f} Kcyc  {100 * v / top.sum():5.1f}%")
