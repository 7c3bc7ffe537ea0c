"""Diagnostic: GPU vs oracle contact sets on random folded-arm states (the self-collision parity states).
Counts, per pair category, contacts present in one and not the other, and the distance differences of the
shared ones.  usage: python tools/dev/contact_set_diff.py [n_states]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-so100-c_amd")]
import torch
from gym_so100 import SO100VecEnv
from gym_so100.model import build_model, PAIR_MPR0, PAIR_SELF0, PAIR_BASE0, PAIR_PADLINK0, PAIR_PAD0
from oracle.oracle import Oracle

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
model = build_model()
o64, o32 = Oracle(64), Oracle(32)
rng = np.random.default_rng(17)
lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
d = o64.new_data()
states = []
while len(states) < N:
    arm = rng.uniform(lo_j, hi_j)
    o64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
    for k in range(6):
        d.qpos[k] = arm[k]
    o64.call("so100o_fwd_position", model, d)
    if any(PAIR_SELF0 <= d.con[i].pair < PAIR_PAD0 for i in range(d.ncon)) and not d.ncon_dropped:
        q, v, w, _ = o64.get_state(d)
        states.append(q)
env = SO100VecEnv(N, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True)
env.reset(seed=3)
q = np.array(states, np.float32)
env.set_state(q, np.zeros((N, 12), np.float32), np.zeros((N, 12), np.float32))
env.step(torch.zeros(N, 6, device="cuda"))
torch.cuda.synchronize()
dbg = env.debug.cpu().numpy()
cat = lambda p: "box" if p < PAIR_MPR0 else "boxhull" if p < PAIR_SELF0 else "self" if p < PAIR_BASE0 else "base" if p < PAIR_PADLINK0 else "padlink" if p < PAIR_PAD0 else "pad"
stats = {}
d64, d32 = o64.new_data(), o32.new_data()
for i in range(N):
    # last substep's contact set: the GPU's debug row vs the oracle's after the same step from the same state
    o64.set_state(d64, q[i].astype(np.float64), np.zeros(12), np.zeros(12))
    o32.set_state(d32, q[i].astype(np.float64), np.zeros(12), np.zeros(12))
    o64.env_step(model, d64, 0, np.zeros(6, np.float32))
    o32.env_step(model, d32, 0, np.zeros(6, np.float32))
    g = {int(p): dbg[i, 16 + c] for c, p in enumerate(dbg[i, 48:48 + int(dbg[i, 0])])}
    r = {d64.con[c].pair: d64.con[c].dist for c in range(d64.ncon)}
    r32 = {d32.con[c].pair: d32.con[c].dist for c in range(d32.ncon)}
    for name, A, B in (("gpu", g, r), ("o32", r32, r)):
        for p in set(A) | set(B):
            s = stats.setdefault((name, cat(p)), [0, 0, 0, []])
            if p in A and p in B:
                s[0] += 1; s[3].append(abs(A[p] - B[p]))
            elif p in A:
                s[1] += 1
            else:
                s[2] += 1
print("vs fp64 oracle after one step: (shared, only-in-x, only-in-o64, median|ddist|, max|ddist|)")
for k in sorted(stats):
    s = stats[k]
    dd = np.array(s[3]) if s[3] else np.zeros(1)
    print(f"  {k[0]:4s} {k[1]:8s} shared {s[0]:4d} only-x {s[1]:3d} only-o64 {s[2]:3d}  |ddist| median {np.median(dd):.2e} max {dd.max():.2e}")
