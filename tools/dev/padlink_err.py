"""Diagnostic: qvel error (GPU vs fp64 oracle, and the fp32 oracle's own) on folded-arm states, grouped by
whether the env has pad/link-hull contacts.  usage: python tools/dev/padlink_err.py [n] [solver]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-so100-c_amd")]
import torch
from gym_so100 import SO100VecEnv
from gym_so100.model import build_model, PAIR_SELF0, PAIR_PADLINK0, PAIR_PAD0
from oracle.oracle import Oracle

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
solver = sys.argv[2] if len(sys.argv) > 2 else "newton"
model = build_model(solver=solver)
o64, o32 = Oracle(64), Oracle(32)
rng = np.random.default_rng(17)
lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
d = o64.new_data()
states, haspl = [], []
while len(states) < N:
    arm = rng.uniform(lo_j, hi_j)
    o64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
    for k in range(6):
        d.qpos[k] = arm[k]
    o64.call("so100o_fwd_position", model, d)
    pairs = [d.con[i].pair for i in range(d.ncon)]
    if any(PAIR_SELF0 <= p < PAIR_PAD0 for p in pairs) and not d.ncon_dropped:
        states.append(o64.get_state(d)[0])
        haspl.append(any(PAIR_PADLINK0 <= p < PAIR_PAD0 for p in pairs))
env = SO100VecEnv(N, device="cuda:0", autoreset=False, max_episode_steps=0, solver=solver)
env.reset(seed=3)
q = np.array(states, np.float32)
env.set_state(q, np.zeros((N, 12), np.float32), np.zeros((N, 12), np.float32))
env.step(torch.zeros(N, 6, device="cuda"))
torch.cuda.synchronize()
gv = env.qvel.cpu().numpy()
d64, d32 = o64.new_data(), o32.new_data()
eg, e32 = [], []
for i in range(N):
    o64.set_state(d64, q[i].astype(np.float64), np.zeros(12), np.zeros(12))
    o32.set_state(d32, q[i].astype(np.float64), np.zeros(12), np.zeros(12))
    o64.env_step(model, d64, 0, np.zeros(6, np.float32))
    o32.env_step(model, d32, 0, np.zeros(6, np.float32))
    ov = o64.get_state(d64)[1]
    eg.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
    e32.append((np.abs(ov - o32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
eg, e32, haspl = np.array(eg), np.array(e32), np.array(haspl)
for name, m in (("with pad-link", haspl), ("without", ~haspl)):
    if m.sum():
        print(f"{solver} {name:14s} n={m.sum():3d}  GPU median {np.median(eg[m]):.2e} p90 {np.quantile(eg[m], .9):.2e} "
              f"max {eg[m].max():.2e} | fp32 oracle median {np.median(e32[m]):.2e} p90 {np.quantile(e32[m], .9):.2e} max {e32[m].max():.2e}")
