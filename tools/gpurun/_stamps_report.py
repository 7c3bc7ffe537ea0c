"""Diagnostic: per-phase cycle attribution of the PGS kernel (last substep), grouped by the wave's max
contact count, and QCQP Newton steps per env (stamps build via SO100_LIB)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = SO100VecEnv(n, device="cuda:0", debug=True)
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for i in range(60):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
torch.cuda.synchronize()
D = []
for i in range(3):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    D.append(env.debug.cpu().numpy())
d = np.concatenate(D)
ncon = d[:, 0].astype(int)
wmax = np.repeat(ncon.reshape(-1, 16).max(1), 16)
st = d[:, 88:93]
newton = d[:, 93]
names = ["record load", "friction+limits", "contacts (resident)", "contacts (overflow)", "tail"]
print("all waves: " + ", ".join(f"{k} {v / 1e3:.1f}K" for k, v in zip(names, st[::16].mean(0))))
for k in range(0, 17):
    m = wmax == k
    if m.sum() == 0:
        continue
    w = st[m][::16].mean(0)
    per_contact = (w[2] + w[3]) / max(k, 1) / 100
    print(f"wave-max ncon {k:2d}: {m.sum() // 16:5d} waves | " + " ".join(f"{v / 1e3:7.1f}K" for v in w) +
          f" | {per_contact:6.0f} cyc/contact-sweep | newton/env {newton[m].mean():8.0f}")
print("newton steps per (contact, sweep) by env ncon:")
for k in range(1, 17):
    m = ncon == k
    if m.sum():
        print(f"  ncon {k:2d}: {m.sum():6d} envs, newton per env {newton[m].mean():8.0f} -> per contact-sweep {newton[m].mean() / k / 100:.2f}")
