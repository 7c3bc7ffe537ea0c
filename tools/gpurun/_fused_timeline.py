"""Fused-kernel wave timeline (diagnostic; needs the -DSO100_TIMELINE library variant via SO100_LIB).

usage: SO100_LIB=.../libso100_hip_timeline.so python tools/gpurun/_fused_timeline.py N [out.npz]
(out.npz: wave durations and start times of 4 consecutive steps)
Each wave's lane-0 env records s_memrealtime (100 MHz) at kernel entry and exit plus HW_ID / XCC_ID in the
debug row (slots 88..93).  Prints the launch span, wave durations, and how many waves were resident at once.
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-so100-c_amd"))
import torch
from gym_so100 import SO100VecEnv

n = int(sys.argv[1])
env = SO100VecEnv(n, device="cuda:0", seed=0, debug=True, convex=os.environ.get("CONVEX", "epa"))
env.reset(seed=1000)
g = torch.Generator(device="cuda").manual_seed(0)
hist = []
for i in range(34):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    if i >= 30:
        torch.cuda.synchronize()
        h = env.debug[::4].cpu().numpy().view(np.uint32)
        a0 = h[:, 88].astype(np.uint64) | (h[:, 89].astype(np.uint64) << 32)
        a1 = h[:, 90].astype(np.uint64) | (h[:, 91].astype(np.uint64) << 32)
        hist.append(((a1 - a0).astype(np.float64) * 0.01, (a0 - a0.min()).astype(np.float64) * 0.01))
torch.cuda.synchronize()
if len(sys.argv) > 2:
    np.savez(sys.argv[2], dur=np.array([x[0] for x in hist]), start=np.array([x[1] for x in hist]))
d = env.debug[::4].cpu().numpy().view(np.uint32)          # lane-0 env of each wave
t0 = d[:, 88].astype(np.uint64) | (d[:, 89].astype(np.uint64) << 32)
t1 = d[:, 90].astype(np.uint64) | (d[:, 91].astype(np.uint64) << 32)
base = t0.min()
s = (t0 - base).astype(np.float64) * 0.01                 # us
e = (t1 - base).astype(np.float64) * 0.01
dur = e - s
print(f"envs {n}, waves {len(s)}, span {e.max():.1f} us, start spread {s.max():.1f} us")
q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
print("wave duration us  min/p10/p50/p90/p99/max:", " ".join(f"{x:.1f}" for x in q))
print("mean duration %.1f us, sum of durations / span = mean resident waves %.0f" % (dur.mean(), dur.sum() / e.max()))
ts = np.linspace(0, e.max(), 41)[:-1]
conc = [int(((s <= t) & (e > t)).sum()) for t in ts]
print("resident waves over the span (40 samples):", conc)
ncon = env.debug[:, 0].cpu().numpy().reshape(-1, 4).max(1)     # wave max contacts, last substep
iters = env.debug[:, 1].cpu().numpy().reshape(-1, 4).max(1)    # wave max Newton iterations, last substep
dd = env.debug[::4].cpu().numpy()
asm, newt, fin = dd[:, 92], dd[:, 93], dd[:, 94]
tot = asm + newt + fin
print("shader kcycles per wave (mean): assembly %.0f  newton %.0f  epilogue %.0f" % (asm.mean() / 1e3, newt.mean() / 1e3, fin.mean() / 1e3))
order = np.argsort(dur)
for name, idx in (("fastest 10%", order[: len(order) // 10]), ("median 10%", order[len(order) * 45 // 100: len(order) * 55 // 100]),
                  ("slowest 1%", order[-max(1, len(order) // 100):])):
    print(f"  {name:12s} dur {dur[idx].mean():7.1f} us  asm {asm[idx].mean()/1e3:6.0f}k newton {newt[idx].mean()/1e3:6.0f}k "
          f"epi {fin[idx].mean()/1e3:5.0f}k  ncon(last) {ncon[idx].mean():4.1f}  iters(last) {iters[idx].mean():4.1f}")
print("start-time quantiles us:", np.percentile(s, [0, 25, 50, 75, 90, 100]).round(1).tolist())
# the slowest waves one by one: per-phase kcycles and each env's last-substep contacts / Newton iterations / pairs
dbg_all = env.debug.cpu().numpy()
for w in np.argsort(dur)[-5:][::-1]:
    envs = range(4 * w, min(4 * w + 4, n))
    desc = "; ".join(f"env {e}: ncon {int(dbg_all[e, 0])} it {int(dbg_all[e, 1])} pairs "
                     f"{[int(p) for p in dbg_all[e, 48:48 + int(dbg_all[e, 0])]]}" for e in envs)
    print(f"wave {w}: {dur[w]:.0f} us, asm {asm[w] / 1e3:.0f}k newton {newt[w] / 1e3:.0f}k | {desc}")
