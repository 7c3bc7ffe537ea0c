"""The oracle's GJK + EPA mesh collider (MuJoCo 3.3.3's default native convex collider) against
an independent exact minimum penetration, on every kind of mesh pair: the cube and the bin boxes against the
link hulls, hull-hull self-collision, the Base hull, the finger pads against link hulls.

The exact minimum penetration of two convex polytopes A (geom1) and B (geom2) is the facet of their Minkowski
difference A - B nearest the origin (scipy ConvexHull of every vertex difference; a box is its 8 corners):
its distance is the depth, its outward normal the direction B must move to separate (geom1 -> geom2).  EPA
converges to that facet to ccd_tolerance (1e-6).  States: random arm poses, the cube dropped near the arm
(tools/dev/mpr_vs_epa.py measures libccd's MPR against the same reference: 29 % of its rollout contacts have
normals more than 5 deg off).
"""
import math

import numpy as np
import pytest
from scipy.spatial import ConvexHull

from gym_so100.model import PAIR_MPR0, PAIR_SELF0, PAIR_BASE0, PAIR_PADLINK0, PAIR_PAD0, build_model


def _points(m, d, g):
    if g >= 0:
        R = np.array(d.geom_xmat[g][:]).reshape(3, 3)
        h = np.array(m.geom_size[g][:])
        s = np.array([[a, b, c] for a in (-1, 1) for b in (-1, 1) for c in (-1, 1)], dtype=float)
        return (s * h) @ R.T + np.array(d.geom_xpos[g][:])
    k = -1 - g
    b = m.hull_body[k]
    R = np.array(d.xmat[b][:]).reshape(3, 3)
    s, n = m.hull_start[k], m.hull_count[k]
    return np.array([m.hull_vert[s + i][:] for i in range(n)]) @ R.T + np.array(d.xpos[b][:])


def _exact(A, B):
    """(depth, normal) of the minimum penetration, and every facet's (distance, normal) for tie checks"""
    eq = ConvexHull((A[:, None, :] - B[None, :, :]).reshape(-1, 3)).equations
    dist = -eq[:, 3]
    f = int(np.argmin(dist))
    return dist[f], eq[f, :3], dist, eq[:, :3]


@pytest.fixture(scope="module")
def epa_contacts(oracle64):
    m = build_model(convex="epa")
    d = oracle64.new_data()
    rng = np.random.default_rng(29)
    lo = np.array([r[0] for r in m.jnt_range]); hi = np.array([r[1] for r in m.jnt_range])
    out = []
    while len(out) < 240:
        arm = rng.uniform(lo, hi)
        oracle64.reset(m, d, np.array([rng.uniform(-0.45, -0.15), rng.uniform(0.35, 0.75), rng.uniform(0.01, 0.2),
                                       1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", m, d)
        for i in range(d.ncon):
            c = d.con[i]
            if PAIR_MPR0 <= c.pair < PAIR_PAD0:
                A, B = _points(m, d, m.pair_geom1[c.pair]), _points(m, d, m.pair_geom2[c.pair])
                out.append((c.pair, -c.dist, np.array(c.frame[:3]), np.array(c.pos[:]), A, B))
    return out


def test_epa_depth_is_the_minimum_penetration(epa_contacts):
    classes = set()
    for p, depth, n, pos, A, B in epa_contacts:
        ex, _, _, _ = _exact(A, B)
        assert abs(depth - ex) <= 1e-6, (p, depth, ex)           # EPA stops within ccd_tolerance
        classes.add("box-hull" if p < PAIR_SELF0 else "self" if p < PAIR_BASE0 else "Base" if p < PAIR_PADLINK0
                    else "pad-link")
    assert classes == {"box-hull", "self", "Base", "pad-link"}


def test_epa_normal_is_a_minimum_penetration_direction(epa_contacts):
    """Along the EPA normal the shapes overlap by exactly the depth (a minimum-penetration direction); it is
    the nearest facet's normal except where facets tie in depth (deep folds)"""
    off, angles = 0, []
    for p, depth, n, pos, A, B in epa_contacts:
        assert abs(np.linalg.norm(n) - 1) < 1e-12
        overlap = (A @ n).max() - (B @ n).min()
        assert abs(overlap - depth) <= 1e-6, (p, overlap, depth)
        ex, en, dist, normals = _exact(A, B)
        ang = math.degrees(math.acos(max(-1.0, min(1.0, float(n @ en)))))
        angles.append(ang)
        if ang > 0.05:
            # then a facet of (nearly) the same depth has this normal (deep folds: facets tie)
            near = normals[dist < ex + 1e-6]
            assert (near @ n).max() > 1 - 1e-6, (p, ang)
            off += 1
    # (EPA stops within ccd_tolerance: on thin facets its normal may lean by ~1e-4 rad)
    assert off <= 0.02 * len(epa_contacts) and np.median(angles) < 1e-4


def test_epa_position_is_between_the_surfaces(epa_contacts):
    """the witness points' midpoint lies within the overlap along the normal, at mid-depth"""
    for p, depth, n, pos, A, B in epa_contacts:
        lo_b, hi_a = (B @ n).min(), (A @ n).max()
        assert lo_b - 1e-9 <= pos @ n <= hi_a + 1e-9
        assert abs(pos @ n - 0.5 * (lo_b + hi_a)) < 1e-6 + 1e-3 * depth


@pytest.mark.parametrize("bits", [64, 32])
def test_separation_cache_changes_nothing(bits):
    """The kernels' separating-direction cache (so100_convex.h mpr_contacts: a convex pair's last separating direction,
    re-checked with one support before GJK) restated in the oracle (so100o_data.sep_on): random-action rollouts with
    and without it are bitwise the same, state and contact lists, in both precisions, while the cache skips most of
    the GJK runs of separated pairs."""
    from oracle.oracle import Oracle
    o = Oracle(bits)
    m = build_model()
    rng = np.random.default_rng(11)
    hits = seps = 0
    for env in range(10):
        pose = o.spawn_pose(100 + env)
        da, db = o.new_data(), o.new_data()
        for d in (da, db):
            o.reset(m, d, pose)
        db.sep_on = 1
        act = rng.uniform(-1, 1, 6).astype(np.float32)
        for step in range(80):
            if step % 8 == 0:
                act = rng.uniform(-1, 1, 6).astype(np.float32)
            for d in (da, db):
                o.env_step(m, d, 0, act)
            for xa, xb in zip(o.get_state(da), o.get_state(db)):
                assert np.array_equal(xa, xb), (env, step)
            pa, pb = o.last_solve(da)[0], o.last_solve(db)[0]
            assert np.array_equal(pa, pb), (env, step)
        hits += db.sep_hits
        seps += db.sep_sep
    print(f"\nGJK runs on separated pairs: {seps} with the cache, {hits} skipped by it")
    assert hits > 2 * seps, (hits, seps)


def test_fp32_collider_matches_fp64_on_folded_poses():
    """The convex collider's fp32 robustness (DESIGN.md §4 deviation 7): on random folded arm poses (self, Base,
    pad-link and box-hull contacts) the fp32 restatement, and the same code with multiply-adds contracted to FMAs
    as the GPU compiler does, find exactly the fp64 contact set with every depth within 1e-5.  Before round 4's
    visibility tolerance an inverted facet (a point on a coplanar facet's plane taken as in front of it) derailed
    fp32 EPA on face-face hull contacts: 3 of 1,200 comparisons (one contact missed, two at half depth)."""
    from oracle.oracle import Oracle
    o64, o32, ofma = Oracle(64), Oracle(32), Oracle(32, fma=True)
    model = build_model()
    rng = np.random.default_rng(5)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    d = o64.new_data()
    n = 0
    while n < 300:
        arm = rng.uniform(lo_j, hi_j)
        o64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        o64.call("so100o_fwd_position", model, d)
        c64 = {d.con[i].pair: d.con[i].dist for i in range(d.ncon) if PAIR_MPR0 <= d.con[i].pair < PAIR_PAD0}
        if not c64:
            continue
        n += 1
        q, v, w, _ = o64.get_state(d)
        for o in (o32, ofma):
            dd = o.new_data()
            o.set_state(dd, q, v, w)
            o.call("so100o_fwd_position", model, dd)
            c = {dd.con[i].pair: dd.con[i].dist for i in range(dd.ncon) if PAIR_MPR0 <= dd.con[i].pair < PAIR_PAD0}
            assert set(c) == set(c64), (n, sorted(set(c) ^ set(c64)))
            assert max(abs(c[p] - c64[p]) for p in c) < 1e-5, n


def test_table_pairs_are_the_minimum_penetration(oracle64):
    """The table is a mesh (scene_so100.xml:3,20), so MuJoCo collides every pair with it through its convex collider:
    one contact at the minimum penetration.  Over random arm poses, including links hanging past the table's edges
    and pushed into its side faces: every arm-hull, finger-pad and cube contact with the table has the exact minimum
    penetration depth (scipy hull of the vertex differences, within 1e-6) and a normal along which the shapes overlap
    by it; a hull or pad overlapping the table has its contact, one not overlapping has none; and side-face contacts
    (normal not vertical) occur for both hulls and pads.  (Before round 5 the hulls took a top-face-only rule and the
    pads a corner rule: 0.57 % of random poses put a hull vertex nearer a side face than the top.)"""
    from gym_so100.model import NPAIR_BOX, NHULL, PAIR_PADBIN0
    PAIR_TABLE = 8                                           # ("red_box", "table"), include/so100_model.h
    m = build_model()
    d = oracle64.new_data()
    rng = np.random.default_rng(17)
    lo = np.array([r[0] for r in m.jnt_range]); hi = np.array([r[1] for r in m.jnt_range])
    table = set(range(NPAIR_BOX, NPAIR_BOX + NHULL)) | set(range(PAIR_PAD0, PAIR_PADBIN0)) | {PAIR_TABLE}
    n = {"hull": 0, "pad": 0, "cube": 0}
    side = {"hull": 0, "pad": 0}
    for _ in range(1000):
        arm = rng.uniform(lo, hi)
        oracle64.reset(m, d, np.array([rng.uniform(-0.62, -0.15), rng.uniform(0.2, 0.75), rng.uniform(-0.005, 0.1),
                                       1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", m, d)
        assert d.ncon_dropped == 0
        got = {}
        for i in range(d.ncon):
            c = d.con[i]
            if c.pair in table:
                assert c.pair not in got                       # one contact per pair
                got[c.pair] = c
        for p in sorted(table):
            g1, g2 = m.pair_geom1[p], m.pair_geom2[p]
            A, B = _points(m, d, g1), _points(m, d, g2)
            if p not in got:
                mov = B if g1 == 0 else A                     # the hull, pad or cube (geom 0 is the table)
                if mov[:, 2].min() < 0:                        # below the top but no contact: no overlap
                    ex, _, _, _ = _exact(A, B)
                    assert ex < 1e-6, (p, ex)
                continue
            c = got[p]
            ex, _, _, _ = _exact(A, B)
            nrm = np.array(c.frame[:3])
            assert abs(-c.dist - ex) <= 1e-6, (p, -c.dist, ex)
            assert abs(((A @ nrm).max() - (B @ nrm).min()) - ex) <= 1e-6, p
            kind = "cube" if p == PAIR_TABLE else "pad" if p >= PAIR_PAD0 else "hull"
            n[kind] += 1
            if kind != "cube" and abs(nrm[2]) < 0.99:
                side[kind] += 1
    print(f"\ntable contacts {n}, side-face contacts {side}")
    assert n["hull"] >= 200 and n["pad"] >= 200 and n["cube"] >= 50, n
    assert side["hull"] >= 5 and side["pad"] >= 5, side


@pytest.mark.parametrize("bits", [64, 32])
def test_top_face_rule_and_collider_agree(bits, oracle64, oracle32):
    """Where the top-face rule applies (a hull over the table's top face, provably its minimum penetration along +z),
    the convex collider gives the same contact (DESIGN.md §3.2 S3a'): GJK + EPA's final facet lies within 1e-5 rad of
    the top face's normal, so the table face snap takes that face's contact, the hull's support vertex along -z and its
    projection, as the rule does.  The kernel decides rule or collider in fp32 and the oracle in fp64, so near the
    rule's bounds the two can take different paths; this pins that the paths agree on depth, normal and
    position, in the fp64 and the fp32 restatement.  so100o_table_force_slow sends every candidate through the
    collider; random arm poses over the table (the generator of test_table_pairs_are_the_minimum_penetration)."""
    import ctypes
    from gym_so100.model import NPAIR_BOX, NHULL
    o = oracle64 if bits == 64 else oracle32
    force = ctypes.c_int.in_dll(o.lib, "so100o_table_force_slow")
    m = build_model()
    d = o.new_data()
    rng = np.random.default_rng(23)
    lo = np.array([r[0] for r in m.jnt_range]); hi = np.array([r[1] for r in m.jnt_range])
    pairs = set(range(NPAIR_BOX, NPAIR_BOX + NHULL))
    tol_pos, tol_depth = (1e-9, 1e-6) if bits == 64 else (2e-6, 2e-6)
    compared = 0
    try:
        for _ in range(600):
            arm = rng.uniform(lo, hi)
            box = np.array([rng.uniform(-0.62, -0.15), rng.uniform(0.2, 0.75), 0.1, 1, 0, 0, 0])
            out = []
            for f in (0, 1):
                force.value = f
                o.reset(m, d, box)
                for k in range(6):
                    d.qpos[k] = arm[k]
                o.call("so100o_fwd_position", m, d)
                out.append({d.con[i].pair: (d.con[i].dist, np.array(d.con[i].frame[:3]), np.array(d.con[i].pos[:]))
                            for i in range(d.ncon) if d.con[i].pair in pairs})
            fast, slow = out
            for p, (dist, nrm, pos) in fast.items():
                if abs(nrm[2] - 1.0) > 0 or p not in slow:
                    continue                      # not a top-face-rule contact (the collider's in both runs), or see below
                sd, sn, sp = slow[p]
                assert abs(sd - dist) <= tol_depth, (p, dist, sd)
                assert np.abs(sn - nrm).max() <= 1e-5, (p, sn)
                assert np.abs(sp - pos).max() <= tol_pos, (p, pos, sp)
                compared += 1
            # every rule contact has its collider twin, and the collider finds no contact the rule missed
            assert set(fast) == set(slow), (sorted(fast), sorted(slow))
    finally:
        force.value = 0
    print(f"\n{bits}-bit: {compared} top-face-rule contacts matched by the collider")
    assert compared >= 100, compared
