"""Newton steps per solve on the GPU (the debug buffer's last-substep iteration count, every env, every step) and the
wave maximum, over a bench-like run (random actions, 8,192 envs by default).  A/B of stop variants via SO100_LIB.
usage: python tools/dev/newton_iters_gpu.py [n_envs] [steps]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
env = SO100VecEnv(n, device="cuda:0", seed=0, debug=True)
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
it, wmax, ncon = [], [], []
for i in range(steps):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    d = env.debug[:, :4].cpu().numpy()
    k = d[:, 1].astype(np.float64)
    it.append(k.mean())
    wmax.append(k.reshape(-1, 4).max(1).mean())
    ncon.append(d[:, 0].mean())
print(f"lib {os.environ.get('SO100_LIB', 'tree')}: envs {n} steps {steps}: Newton steps (last substep) mean "
      f"{np.mean(it):.4f}, wave max mean {np.mean(wmax):.4f}, ncon mean {np.mean(ncon):.3f}")
