"""Evaluate the MPR collider (libccd, the oracle's and the kernel's convex pairs) against the exact minimum
penetration that MuJoCo 3.3.3's default native GJK/EPA converges to (DESIGN.md §4 deviation 7).

For each convex contact the oracle reports on sampled states, the exact minimum penetration of the two
convex shapes is computed from the facets of their Minkowski difference (scipy ConvexHull of all vertex
differences; a box is its 8 corners): depth = min over facets of the facet's distance from the origin,
normal = that facet's outward normal (from geom1 towards geom2 as the oracle's frame).  EPA converges to this
(to its tolerance); MPR reports the penetration along the centre-to-centre ray's portal instead.

usage: python tools/dev/mpr_vs_epa.py [states] [mpr|epa] > report   (the oracle's convex collider to evaluate)
"""
import math
import os
import sys

import numpy as np
from scipy.spatial import ConvexHull

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-so100-c_amd")]
from oracle.oracle import Oracle  # noqa: E402
from gym_so100.model import (PAIR_MPR0, PAIR_SELF0, PAIR_BASE0, PAIR_PADLINK0, PAIR_PAD0, NHULL,  # noqa: E402
                             build_model)


def geom_points(m, d, g):
    """world vertices of geom g: a box's 8 corners (g >= 0) or hull -1-g's vertices"""
    if g >= 0:
        R = np.array(d.geom_xmat[g][:]).reshape(3, 3)
        c = np.array(d.geom_xpos[g][:])
        h = np.array(m.geom_size[g][:])
        corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * h
        return corners @ R.T + c
    k = -1 - g
    b = m.hull_body[k]
    R = np.array(d.xmat[b][:]).reshape(3, 3)
    p = np.array(d.xpos[b][:])
    s, n = m.hull_start[k], m.hull_count[k]
    V = np.array([m.hull_vert[s + i][:] for i in range(n)])
    return V @ R.T + p


def exact_penetration(A, B):
    """minimum translation separating A and B (both point sets' hulls): depth and unit normal n such that
    moving B by depth * n separates them (n points from A towards B)"""
    D = (A[:, None, :] - B[None, :, :]).reshape(-1, 3)        # Minkowski difference A - B
    hull = ConvexHull(D)
    eq = hull.equations                                       # n . x + off <= 0 inside, |n| = 1
    dist = -eq[:, 3]                                          # distance of each facet plane from the origin
    if (dist < 0).any():
        return None                                           # origin outside: no penetration
    f = np.argmin(dist)
    return dist[f], eq[f, :3]        # B moving by depth along A - B's outward facet normal separates them


COLLIDER = sys.argv[2] if len(sys.argv) > 2 else "mpr"


def _oracle():
    return Oracle(64)


def main():
    nstates = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    o = _oracle()
    m = build_model(convex=COLLIDER)
    d = o.new_data()
    rng = np.random.default_rng(7)
    lo = np.array([r[0] for r in m.jnt_range])
    hi = np.array([r[1] for r in m.jnt_range])
    res = {}
    got = 0
    while got < nstates:
        arm = rng.uniform(lo, hi)
        # the cube on a random spot near the arm, for box-hull pairs too
        o.reset(m, d, np.array([rng.uniform(-0.45, -0.15), rng.uniform(0.35, 0.75), rng.uniform(0.01, 0.2), 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        o.call("so100o_fwd_position", m, d)
        cons = [d.con[i] for i in range(d.ncon) if PAIR_MPR0 <= d.con[i].pair < PAIR_PAD0]
        if not cons:
            continue
        got += 1
        for c in cons:
            p = c.pair
            cls = ("box-hull" if p < PAIR_SELF0 else "self" if p < PAIR_BASE0 else "Base" if p < PAIR_PADLINK0
                   else "pad-link")
            g1, g2 = m.pair_geom1[p], m.pair_geom2[p]
            r = exact_penetration(geom_points(m, d, g1), geom_points(m, d, g2))
            e = res.setdefault(cls, {"n": 0, "ang": [], "ddep": [], "depth": [], "miss": 0})
            e["n"] += 1
            if r is None:
                e["miss"] += 1
                continue
            depth, n = r
            nm = np.array(c.frame[:3])
            e["ang"].append(math.degrees(math.acos(max(-1.0, min(1.0, float(nm @ n))))))
            e["ddep"].append(-c.dist - depth)
            e["depth"].append(depth)
    print(f"{nstates} random arm poses with convex contacts; the oracle's {COLLIDER.upper()} (fp64) vs the exact minimum "
          "penetration")
    for cls, e in res.items():
        a, dd, dep = np.array(e["ang"]), np.array(e["ddep"]), np.array(e["depth"])
        print(f"{cls:9s} contacts {e['n']:5d} (no overlap in the exact test: {e['miss']}) | normal angle deg: median "
              f"{np.median(a):.3g} p90 {np.quantile(a, .9):.3g} max {a.max():.3g}, share > 5 deg {np.mean(a > 5):.3f} | "
              f"depth - exact depth (m): median {np.median(dd):.2e} p90 {np.quantile(dd, .9):.2e} max {dd.max():.2e} "
              f"| exact depth median {np.median(dep):.2e} | share with |depth error| > 10 %: "
              f"{np.mean(np.abs(dd) > 0.1 * dep):.3f}")




def rollout_eval(nenv=96, steps=300):
    """the same comparison on the bench's workload: random-action rollouts from RandomState spawns"""
    o = _oracle()
    m = build_model(convex=COLLIDER)
    rng = np.random.default_rng(11)
    res = {}
    for e in range(nenv):
        d = o.new_data()
        o.reset(m, d, o.spawn_pose(1000 + e))
        for s in range(steps):
            o.env_step(m, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
            o.call("so100o_fwd_position", m, d)
            for i in range(d.ncon):
                c = d.con[i]
                if not PAIR_MPR0 <= c.pair < PAIR_PAD0:
                    continue
                p = c.pair
                cls = ("box-hull" if p < PAIR_SELF0 else "self" if p < PAIR_BASE0 else "Base" if p < PAIR_PADLINK0
                       else "pad-link")
                r = exact_penetration(geom_points(m, d, m.pair_geom1[p]), geom_points(m, d, m.pair_geom2[p]))
                x = res.setdefault(cls, {"ang": [], "ddep": [], "depth": [], "miss": 0})
                if r is None:
                    x["miss"] += 1
                    continue
                depth, n = r
                x["ang"].append(math.degrees(math.acos(max(-1.0, min(1.0, float(np.array(c.frame[:3]) @ n))))))
                x["ddep"].append(-c.dist - depth)
                x["depth"].append(depth)
    print(f"random-action rollouts ({nenv} envs x {steps} steps): convex contacts, {COLLIDER.upper()} vs the exact minimum "
          "penetration")
    for cls, x in res.items():
        a, dd, dep = np.array(x["ang"]), np.array(x["ddep"]), np.array(x["depth"])
        if not len(a):
            continue
        print(f"{cls:9s} contacts {len(a):5d} | normal angle deg: median {np.median(a):.3g} p90 {np.quantile(a, .9):.3g} "
              f"max {a.max():.3g}, share > 5 deg {np.mean(a > 5):.3f} | depth error median {np.median(dd):.2e} p90 "
              f"{np.quantile(dd, .9):.2e} | exact depth median {np.median(dep):.2e}")


if __name__ == "__main__":
    main()
    rollout_eval()
