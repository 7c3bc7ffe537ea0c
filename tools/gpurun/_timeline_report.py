"""Diagnostic: per-wave timeline of the last PGS launch of a step (timeline build via SO100_LIB)."""
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
for rep in range(3):
    env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    d = env.debug.cpu().numpy()[::16]
    raw = d[:, 92:96].copy().view(np.uint32)
    t0, t1, hw, misc = raw[:, 0].astype(np.int64), raw[:, 1].astype(np.int64), raw[:, 2], raw[:, 3]
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0          # us (100 MHz)
    dur = e - s
    nmax = misc & 0xFF
    xcc = (misc >> 8) & 0xFF
    print(f"launch span {e.max():.0f} us, waves {len(s)}; wave duration us: p50 {np.median(dur):.0f} p90 {np.quantile(dur,.9):.0f} p99 {np.quantile(dur,.99):.0f} max {dur.max():.0f}")
    for k in range(0, 17):
        m = nmax == k
        if m.sum():
            print(f"   wave-max ncon {k:2d}: {m.sum():5d} waves, dur mean {dur[m].mean():6.0f} max {dur[m].max():6.0f}, start mean {s[m].mean():6.0f}")
    last = np.argsort(e)[-5:]
    print("   last-finishing waves (start, dur, ncon_max, xcc):", [(int(s[i]), int(dur[i]), int(nmax[i]), int(xcc[i])) for i in last])
    st = np.sort(s)
    print("   start-time quantiles us:", [int(x) for x in np.quantile(st, [0, .25, .5, .75, .9, 1])])
    busy = np.bincount(xcc, weights=dur, minlength=8)
    print("   per-XCC wave-us:", [int(x) for x in busy[:8]])
