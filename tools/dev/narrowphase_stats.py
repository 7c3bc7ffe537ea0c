"""Convex-narrowphase statistics on the bench workload (dev probe, CPU): per position stage of the fp32 oracle
built with -DSO100O_STATS, the broadphase candidates, GJK overlaps, EPA contacts and GJK / EPA iterations; per
4-env wave (consecutive env ids, as the kernel groups them) the rounds the shared narrowphase runs.

    cc -O2 -fPIC -std=c11 -I include -DSO100O_FLOAT -DSO100O_STATS -shared -o /tmp/liboracle32_stats.so \
        oracle/so100_oracle.c -lm
    python tools/dev/narrowphase_stats.py [nenv] [steps]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
from oracle.oracle import Oracle  # noqa: E402
from gym_so100.model import build_model  # noqa: E402


def main():
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    o = Oracle(32)
    lib = ctypes.CDLL("/tmp/liboracle32_stats.so")
    lib.so100o_batch_run.argtypes = o.lib.so100o_batch_run.argtypes
    lib.so100o_batch_run.restype = ctypes.c_long
    lib.so100o_reset.argtypes = o.lib.so100o_reset.argtypes
    lib.so100o_stats_reset.argtypes = [ctypes.c_void_p, ctypes.c_long]
    lib.so100o_stats_count.restype = ctypes.c_long
    lib.so100o_items_reset.argtypes = [ctypes.c_void_p, ctypes.c_long]
    lib.so100o_items_count.restype = ctypes.c_long
    o.lib = lib
    m = build_model()
    datas = (o.Data * nenv)()
    for i in range(nenv):
        o.reset(m, datas[i], o.spawn_pose(1000 + i))
    rng = np.random.default_rng(0)
    per_step = m.nsubstep + 1
    warm = 10
    for s in range(warm):                                    # past the initial drop
        o.batch_run(m, datas, nenv, 1, 0, rng.uniform(-1, 1, (1, nenv, 6)).astype(np.float32), nthreads=1)
    buf = np.zeros((steps * nenv * per_step + 16, 5), np.int64)
    lib.so100o_stats_reset(buf.ctypes.data, len(buf))
    items = np.zeros((4 << 20, 4), np.int64)
    lib.so100o_items_reset(items.ctypes.data, len(items))
    for s in range(steps):
        o.batch_run(m, datas, nenv, 1, 0, rng.uniform(-1, 1, (1, nenv, 6)).astype(np.float32), nthreads=1)
    item_report(items[:min(lib.so100o_items_count(), len(items))])
    n = lib.so100o_stats_count()
    assert n == steps * nenv * per_step, (n, steps * nenv * per_step)
    st = buf[:n].reshape(steps, nenv, per_step, 5)[:, :, :m.nsubstep]   # the substeps' position stages
    cand, ovl, hit, gjk, epa = (st[..., k] for k in range(5))
    print(f"{nenv} envs x {steps} steps x {m.nsubstep} substeps: per env-substep mean candidates {cand.mean():.3f}, "
          f"GJK overlaps {ovl.mean():.3f}, contacts {hit.mean():.3f}; GJK iterations per candidate "
          f"{gjk.sum() / max(cand.sum(), 1):.2f}, EPA iterations per overlap {epa.sum() / max(ovl.sum(), 1):.2f}")
    print("env-substeps with candidates: %.4f; with > 8: %.5f" % ((cand > 0).mean(), (cand > 8).mean()))
    # per wave (4 consecutive envs) and substep: rounds now (all candidates) vs split (GJK all, EPA overlaps)
    w = nenv // 4
    wc = cand[:, :4 * w].reshape(steps, w, 4, m.nsubstep).sum(2)
    wo = ovl[:, :4 * w].reshape(steps, w, 4, m.nsubstep).sum(2)
    r_now = np.ceil(wc / 4)
    r_gjk, r_epa = np.ceil(wc / 4), np.ceil(wo / 4)
    for q in (50, 90, 99, 99.9, 100):
        print(f"  wave-substep p{q}: candidates {np.percentile(wc, q):.0f}, overlaps {np.percentile(wo, q):.0f}, "
              f"rounds now {np.percentile(r_now, q):.0f}, EPA rounds if split {np.percentile(r_epa, q):.0f}")
    # per wave and env step (10 substeps): the heavy tail the step waits for
    sc, so = wc.sum(2), wo.sum(2)
    top = np.argsort(sc.ravel())[-max(1, sc.size // 100):]
    print(f"slowest-1% wave-steps by candidates: candidates {sc.ravel()[top].mean():.1f}, overlaps {so.ravel()[top].mean():.1f} "
          f"per step (10 substeps); all: {sc.mean():.2f} / {so.mean():.2f}")


def item_report(items):
    gi, ei, hit = items[:, 0], items[:, 1], items[:, 3]
    ov = ei > 0
    print(f"{len(items)} narrowphase items: GJK iterations p50/p90/p99/max {np.percentile(gi, [50, 90, 99, 100])}, "
          f"EPA iterations (overlapping items) p50/p90/p99/max {np.percentile(ei[ov], [50, 90, 99, 100]) if ov.any() else '-'}")
    sep = items[:, 2] > 0
    print(f"  box-axis SAT (hull's exact projection on the box's 3 face axes) separates {sep.mean():.3f} of all items, "
          f"{sep[~ov].mean() if (~ov).any() else 0:.3f} of the GJK-separated ones (GJK iterations saved "
          f"{gi[sep].sum() / max(gi.sum(), 1):.3f}); overlapping items it separates: {int((sep & ov).sum())}")
    print("  GJK iteration histogram:", np.bincount(gi, minlength=8)[:51].tolist())
    print("  EPA iteration histogram:", np.bincount(ei[ov], minlength=8)[:51].tolist() if ov.any() else [])


if __name__ == "__main__":
    main()
