"""Diagnostic: per-phase cycles of the stage kernel (mode 1, last substep); stage-stamps build via SO100_LIB.
usage: SO100_LIB=<stamps build> python tools/gpurun/_stage_stamps_report.py [solver] [n] [dyn]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
env = SO100VecEnv(n, device="cuda:0", debug=True, solver=sys.argv[1] if len(sys.argv) > 1 else "newton",
                  convex=os.environ.get("CONVEX", "epa"))
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for i in range(60):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
acc = np.zeros(8)
rows = []
for i in range(3):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    acc += env.debug.cpu().numpy()[::4, 88:96].mean(0)
    rows.append(env.debug.cpu().numpy()[::4, 88:96])
acc /= 3
names = ["Euler", "S1-S2 FK + dynamics", "S3c box-box + compaction", "S6a J + reductions", "S6b per-contact setup",
         "S7 + record", "S3a hulls vs table", "S3b box-hull MPR"]
if len(sys.argv) > 3 and sys.argv[3] == "dyn":     # -DSO100_DYN_STAMPS build: the S1-S2 phases
    names = ["sincos", "FK chain (lane 0)", "comPos", "CRBA", "Cholesky (lane 0)", "M^-1 + RNE velocities",
             "RNE forces", "bias + qacc_smooth"]
for k, v in zip(names, acc):
    print(f"{k:24s} {v / 1e3:8.1f} Kcyc  {100 * v / acc.sum():5.1f}%")
R = np.concatenate(rows)
top = R[np.argsort(R.sum(1))[-max(1, len(R) // 100):]].mean(0)
print("slowest 1% of waves:")
for k, v in zip(names, top):
    print(f"{k:26s} {v / 1e3:8.1f} Kcyc  {100 * v / top.sum():5.1f}%")
