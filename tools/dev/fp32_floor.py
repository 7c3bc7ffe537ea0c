"""The fp32 floor of the deep-fold parity states on the CPU: the fp32 restatement, host-compiled and with FMA
contraction (liboracle32fma, as the GPU compiler contracts), teacher-forced from the fp64 trajectory on
_arm_contact_parity's states (test-side tool; no GPU).

    python tools/dev/fp32_floor.py base|padlink|overflow
"""
import sys, numpy as np
ROOT = __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
sys.path[:0] = [ROOT + '/gym-so100-c_amd', ROOT, ROOT + '/tests']
from oracle.oracle import Oracle
from gym_so100.model import build_model, PAIR_BASE0, PAIR_PADLINK0, PAIR_MOCAPHULL0, NPAIR
o64, o32, ofma = Oracle(64), Oracle(32), Oracle(32, fma=True)
which = sys.argv[1]
cfg = {"base": (PAIR_BASE0, PAIR_PADLINK0, 19, None, None), "padlink": (PAIR_PADLINK0, PAIR_MOCAPHULL0, 23, None, None),
       "overflow": (0, NPAIR, 29, None, lambda d: d.ncon > 16)}[which]
p0, p1, seed, nsub, select = cfg
model = build_model(solver="newton", nsubstep=nsub)
rng = np.random.default_rng(seed)
lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
d = o64.new_data(); states, targets = [], []
while len(states) < 48:
    arm = rng.uniform(lo_j, hi_j)
    o64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
    for k in range(6): d.qpos[k] = arm[k]
    o64.call("so100o_fwd_position", model, d)
    if (select(d) if select else any(p0 <= d.con[i].pair < p1 for i in range(d.ncon))) and not d.ncon_dropped:
        q, v, w, _ = o64.get_state(d); states.append((q, v * 0, w * 0)); targets.append(np.clip((arm - lo) / (hi - lo) * 2 - 1, -1, 1))
targets = np.array(targets)
def rel(a, b): return np.abs(a - b).max() / max(1.0, np.abs(b).max())
e32, efma = [], []
cur = [o64.new_data() for _ in states]
for i, s in enumerate(states): o64.set_state(cur[i], *s)
for step in range(3):
    act = (targets + rng.normal(0, 0.02, targets.shape)).astype(np.float32)
    for i in range(48):
        q, v, w = [x.astype(np.float32).astype(np.float64) for x in o64.get_state(cur[i])[:3]]
        ref = o64.new_data(); o64.set_state(ref, q, v, w); o64.env_step(model, ref, 0, act[i]); ov = o64.get_state(ref)[1]
        for o, acc in ((o32, e32), (ofma, efma)):
            dd = o.new_data(); o.set_state(dd, q, v, w); o.env_step(model, dd, 0, act[i]); acc.append(rel(o.get_state(dd)[1], ov))
        o64.set_state(cur[i], q, v, w); o64.env_step(model, cur[i], 0, act[i])
for name, e in (("fp32", e32), ("fp32 fma", efma)):
    e = np.array(e); print(f"{which} {name}: qvel rel median {np.median(e):.2e} p90 {np.quantile(e,.9):.2e} p99 {np.quantile(e,.99):.2e} max {e.max():.2e}")
