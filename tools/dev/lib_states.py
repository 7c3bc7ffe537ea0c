"""Dev probe: step N envs K times with random actions through the library SO100_LIB names and save the final
state (qpos, qvel, warmstart, obs, reward, contact bits) to an .npz, so two builds can be compared bit for bit.
usage: SO100_LIB=<lib> python tools/dev/lib_states.py N K out.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-so100-c_amd"))
import torch  # noqa: E402
from gym_so100 import SO100VecEnv  # noqa: E402

n, k, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
env = SO100VecEnv(n, device="cuda:0", seed=0)
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(k):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
torch.cuda.synchronize()
np.savez(out, qpos=env.qpos.cpu().numpy(), qvel=env.qvel.cpu().numpy(), warm=env.qacc_warmstart.cpu().numpy(),
         obs=env.obs.cpu().numpy(), reward=env.reward.cpu().numpy(), bits=env.contact_bits.cpu().numpy())
print("saved", out, "build", env.fused_build)
