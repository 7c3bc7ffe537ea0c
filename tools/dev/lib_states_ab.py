"""Dev probe: the state after a few steps of one library (SO100_LIB), saved for a bitwise comparison with another.
usage: SO100_LIB=... python tools/dev/lib_states_ab.py out.npz [n] [steps] [debug]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv
out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
env = SO100VecEnv(n, device="cuda:0", seed=0, debug=len(sys.argv) > 4)
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
qs = []
for i in range(steps):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    qs.append(env.qpos.cpu().numpy().copy())
np.savez(out, q=np.array(qs))
