"""Dev diagnostic (GPU): first-substep contact sets of the HIP stage kernel vs the fp64/fp32 oracle on
oracle-generated states with box-hull (MPR) contacts."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gym-so100-c_amd"), ROOT]
import numpy as np
import torch
from gym_so100 import vec_env
from gym_so100.model import build_model, PAIR_MPR0
from oracle.oracle import Oracle

m = build_model()
o64, o32 = Oracle(64), Oracle(32)
rng = np.random.default_rng(21)
d = o64.new_data()
states = []
for e in range(64):
    o64.reset(m, d, o64.spawn_pose(2000 + e))
    for _ in range(200):
        o64.env_step(m, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
        if any(d.con[i].pair >= PAIR_MPR0 for i in range(d.ncon)) and not d.ncon_dropped:
            states.append(o64.get_state(d)[:3]); break
    if len(states) >= 32: break
n = len(states)
orig = vec_env.build_model
vec_env.build_model = lambda iterations=None: orig(iterations=iterations, nsubstep=1)
env = vec_env.SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True)
env.reset(seed=3)
Q = np.array([s[0] for s in states], np.float32); V = np.array([s[1] for s in states], np.float32)
W = np.array([s[2] for s in states], np.float32)
env.set_state(Q, V, W)
act = rng.uniform(-1, 1, (n, 6)).astype(np.float32)
env.step(torch.from_numpy(act).cuda()); torch.cuda.synchronize()
dbg = env.debug.cpu().numpy()
m1 = build_model(nsubstep=1)
for i in range(n):
    out = []
    for o in (o64, o32):
        dd = o.new_data()
        o.set_state(dd, Q[i].astype(np.float64), V[i].astype(np.float64), W[i].astype(np.float64))
        o.call("so100o_fwd_position", m1, dd)
        out.append([(dd.con[c].pair, dd.con[c].dist) for c in range(dd.ncon)])
    g = [(int(dbg[i, 48 + c]), float(dbg[i, 16 + c])) for c in range(int(dbg[i, 0]))]
    same = [p for p, _ in g] == [p for p, _ in out[0]]
    dmax = max([abs(a[1] - b[1]) for a, b in zip(g, out[0])] + [0]) if same else -1
    print(i, "same" if same else "DIFF", f"dist maxdiff {dmax:.2e}", "gpu", [(p, f"{x:.5f}") for p, x in g if p >= 23],
          "o64", [(p, f"{x:.5f}") for p, x in out[0] if p >= 23], "o32", [(p, f"{x:.5f}") for p, x in out[1] if p >= 23])
