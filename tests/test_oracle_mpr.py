"""Box vs convex hull contacts through the convex collider (pairs 23..76: the cube and the bin boxes
against every arm/jaw hull) in the oracle, with both colliders the model offers: GJK + EPA
(so100_model.convex = SO100_CONVEX_EPA, MuJoCo 3.3.3's default native collider: the minimum penetration) and
libccd's MPR (SO100_CONVEX_MPR, MuJoCo's mjDSBL_NATIVECCD path: the penetration along the centres' ray).

MuJoCo is not in this container, so the expected values are restated, not MuJoCo's own:
  * a known answer: a box-shaped "hull" overlapping an aligned cube by delta along one axis;
  * on the model's real hulls, against an independent numpy separating-axis evaluation of the same
    polytopes: MPR reports a contact exactly when the shapes overlap, its depth is never below the
    minimum penetration depth, and the contact plane (normal, depth) supports the Minkowski
    difference (the property libccd's MPR terminates on);
  * the constraint rows the contacts make (condim 4 with cube and arm dofs for the cube, condim 3 on
    arm dofs only for the bin boxes).
"""
import copy

import numpy as np
import pytest
from scipy.spatial import ConvexHull

from gym_so100.model import NHULL, PAIR_MPR0, PAIR_PAD0, PAIR_BASE0, build_model


@pytest.fixture(params=["epa", "mpr"], scope="module")
def model(request):
    """this module's tests run with each convex collider"""
    m = build_model(convex=request.param)
    m.convex_name = request.param
    return m

NV = 12
CUBE_HALF = 0.02


def _hull(model, k):
    s, n = model.hull_start[k], model.hull_count[k]
    return np.array([[model.hull_vert[s + i][t] for t in range(3)] for i in range(n)])


def _state(o, m, arm, box):
    d = o.new_data()
    o.reset(m, d, np.asarray(box, dtype=np.float64))
    for k in range(6):
        d.qpos[k] = arm[k]
    o.call("so100o_fwd_position", m, d)
    return d


def _mat2quat(R):
    w = np.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.copysign(np.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])) / 2, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])) / 2, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2])) / 2, R[1, 0] - R[0, 1])
    q = np.array([w, x, y, z])
    return q / np.linalg.norm(q)


def _quat2mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _box_corners(c, R, h):
    s = np.array([[a, b, e] for a in (-1, 1) for b in (-1, 1) for e in (-1, 1)], dtype=float)
    return c + (s * h) @ R.T


def _sat(box_pts, R, hull_pts, hull):
    """Exact minimum penetration depth of two convex polytopes (negative: separated) by brute-force SAT
    over face normals and edge-edge cross products."""
    axes = [hull.equations[:, :3], R.T]
    edges = set()
    for simp in hull.simplices:
        for a, b in ((0, 1), (1, 2), (2, 0)):
            edges.add(tuple(sorted((simp[a], simp[b]))))
    e = np.array([hull.points[j] - hull.points[i] for i, j in edges])
    for k in range(3):
        c = np.cross(R[:, k], e)
        n = np.linalg.norm(c, axis=1)
        axes.append(c[n > 1e-9] / n[n > 1e-9, None])
    L = np.concatenate(axes)
    pa, pb = box_pts @ L.T, hull_pts @ L.T
    overlap = np.minimum(pa.max(0) - pb.min(0), pb.max(0) - pa.min(0))
    return overlap.min()


def test_mpr_known_answer_aligned_box_hull(model, oracle64):
    """Hull 0 replaced by a box in its body frame; the cube, aligned with that frame, overlaps it by
    delta along one axis: one contact, dist = -delta, normal from the cube to the hull, position inside
    the overlap's cross-section near its mid-plane."""
    m = copy.deepcopy(model)
    k, half, cH = 0, np.array([0.03, 0.025, 0.035]), np.array([0.01, 0.05, 0.02])
    corners = _box_corners(cH, np.eye(3), half)
    m.hull_count[k] = 8
    for i in range(8):
        for t in range(3):
            m.hull_vert[m.hull_start[k] + i][t] = corners[i, t]
    for t in range(3):
        m.hull_center[k][t] = cH[t]; m.hull_half[k][t] = half[t]; m.hull_centroid[k][t] = cH[t]
    arm = np.array(model.start_qpos[:])
    d0 = _state(oracle64, m, arm, (0.4, 0.95, 0.6, 1, 0, 0, 0))
    b = m.hull_body[k]
    RH, pH = np.array(d0.xmat[b][:]).reshape(3, 3), np.array(d0.xpos[b][:])
    for axis in range(3):
        for sign in (1.0, -1.0):
            for delta in (1e-3, 4e-3):
                for roll in (0.0, 0.5):          # cube rolled about the contact axis: same depth
                    e = np.zeros(3); e[axis] = sign
                    ca = np.zeros(3); ca[axis] = 1.0
                    Rroll = _quat2mat(np.concatenate([[np.cos(roll / 2)], np.sin(roll / 2) * ca]))
                    Rc = RH @ Rroll
                    off = cH + e * (half[axis] + CUBE_HALF - delta)
                    pos = pH + RH @ off
                    d = _state(oracle64, m, arm, np.concatenate([pos, _mat2quat(Rc)]))
                    got = [d.con[i] for i in range(d.ncon) if d.con[i].pair == PAIR_MPR0 + k]
                    assert len(got) == 1, (axis, sign, delta, roll)
                    c = got[0]
                    assert abs(c.dist + delta) < 1e-9, (c.dist, delta)
                    n = np.array(c.frame[:3])
                    np.testing.assert_allclose(n, -(RH @ e), atol=1e-9)
                    local = RH.T @ (np.array(c.pos[:]) - pH) - cH
                    # libccd's findPos weights the portal's support points by the origin's barycentric
                    # coordinates in the portal tetrahedron (v0 = the centres included): near, not on,
                    # the mid-plane of the overlap
                    assert abs(local[axis] - sign * (half[axis] - delta / 2)) < delta
                    others = [t for t in range(3) if t != axis]
                    assert np.all(np.abs(local[others]) <= half[others] + 1e-9)


def _random_overlaps(model, o, n, seed):
    """Configurations with the cube placed across a hull's surface (random arm pose, hull, vertex,
    offset, cube orientation)."""
    rng = np.random.default_rng(seed)
    lo = np.array([r[0] for r in model.jnt_range]); hi = np.array([r[1] for r in model.jnt_range])
    out = []
    while len(out) < n:
        arm = rng.uniform(lo, hi)
        k = int(rng.integers(NHULL))
        d = _state(o, model, arm, (0.4, 0.95, 0.6, 1, 0, 0, 0))
        b = model.hull_body[k]
        RH, pH = np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])
        v = _hull(model, k)
        w = v @ RH.T + pH
        if w[:, 2].min() < 0.03:                 # keep the cube off the table and the bin out of it
            continue
        p = w[rng.integers(len(w))] + rng.normal(0, 0.012, 3)
        q = rng.normal(size=4)
        out.append((arm, k, np.concatenate([p, q / np.linalg.norm(q)])))
    return out


def test_mpr_matches_separating_axis_geometry(model, oracle64):
    """MPR reports a contact exactly when SAT says the polytopes overlap.  Its depth is the distance from
    the origin to the final portal of the Minkowski difference: never below the true minimum (SAT) depth,
    equal to it for shallow contacts and for most deep ones (MPR approximates the minimum only along its
    centre line), and the shapes still overlap by at least that much along the reported normal."""
    n_miss, ratio, shallow = 0, [], 0
    m_epa = model.convex_name == "epa"
    for arm, k, box in _random_overlaps(model, oracle64, 160, seed=5):
        d = _state(oracle64, model, arm, box)
        b = model.hull_body[k]
        RH, pH = np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])
        hull_w = _hull(model, k) @ RH.T + pH
        hull = ConvexHull(hull_w)
        Rc = _quat2mat(np.array(box[3:]))
        cube_w = _box_corners(np.array(box[:3]), Rc, np.full(3, CUBE_HALF))
        sat = _sat(cube_w, Rc, hull_w, hull)
        got = [d.con[i] for i in range(d.ncon) if d.con[i].pair == PAIR_MPR0 + k]
        if sat < -1e-6:
            assert not got, (k, sat)
            n_miss += 1
            continue
        if sat < 1e-6 or d.ncon_dropped:
            continue                               # touching within the tolerance, or the contact cap hit
        assert len(got) == 1, (k, sat)
        c = got[0]
        depth, nrm = -c.dist, np.array(c.frame[:3])
        assert abs(np.linalg.norm(nrm) - 1) < 1e-12
        assert depth >= sat - 1e-6, (depth, sat)           # MPR / EPA stop within ccd_tolerance
        overlap = (cube_w @ nrm).max() - (hull_w @ nrm).min()
        assert overlap >= depth - 1e-9, (overlap, depth)
        if m_epa:                                           # EPA converges to the minimum penetration itself
            assert abs(depth - sat) < 1e-6 + 1e-6 * sat, (depth, sat)
            assert abs(overlap - depth) < 1e-6 + 1e-6 * sat, (overlap, depth)
        if sat < 2e-3:
            assert abs(depth - sat) < 1e-7 + 1e-4 * sat, (depth, sat)
            shallow += 1
        ratio.append(depth / sat)
        # the position lies between the two shapes' extreme points along the normal
        assert (hull_w @ nrm).min() - 1e-9 <= np.array(c.pos[:]) @ nrm <= (cube_w @ nrm).max() + 1e-9
    # (random arm poses: the pads, the Base and self-collision add contacts, and a few states hit the
    # 16-contact cap and are skipped)
    assert len(ratio) > 80 and n_miss > 5 and shallow >= 3, (len(ratio), n_miss, shallow)
    assert abs(np.median(ratio) - 1) < 0.02, np.median(ratio)


def test_mpr_contact_rows(model, oracle64):
    """Cube-hull contacts: condim 4, J on the cube's and the arm's dofs.  Bin-hull contacts: condim 3, J
    on arm dofs only."""
    kinds = {}
    rng = np.random.default_rng(0)
    for e in range(24):
        d = oracle64.new_data()
        oracle64.reset(model, d, oracle64.spawn_pose(1000 + e))
        for _ in range(150):
            oracle64.env_step(model, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
            if not any(PAIR_MPR0 <= d.con[i].pair < PAIR_PAD0 for i in range(d.ncon)):
                continue
            oracle64.call("so100o_fwd_position", model, d)
            oracle64.call("so100o_fwd_velocity", model, d)
            oracle64.call("so100o_fwd_acceleration", model, d)
            for i in range(d.nefc):
                if d.efc_type[i] != 2 or d.efc_dim[i] == 0:
                    continue
                p = d.con[d.efc_id[i]].pair
                if not PAIR_MPR0 <= p < PAIR_BASE0:
                    continue
                cube = p < PAIR_MPR0 + NHULL
                dim = d.efc_dim[i]
                J = np.array([[d.efc_J[i + r][v] for v in range(NV)] for r in range(dim)])
                assert dim == (4 if cube else 3)
                assert np.abs(J[:3, :6]).max() > 0
                assert (np.abs(J[:, 6:]).max() > 0) == cube
                assert d.efc_force[i] >= 0.0
                kinds[cube] = kinds.get(cube, 0) + 1
    assert kinds.get(True, 0) > 0 and kinds.get(False, 0) > 0, kinds


def _self_configs(model, o, n, seed):
    from gym_so100.model import PAIR_SELF0, PAIR_BASE0
    rng = np.random.default_rng(seed)
    lo = np.array([r[0] for r in model.jnt_range]); hi = np.array([r[1] for r in model.jnt_range])
    hit, miss = [], []
    while len(hit) < n or len(miss) < n:
        arm = rng.uniform(lo, hi)
        d = _state(o, model, arm, (0.4, 0.95, 0.6, 1, 0, 0, 0))
        pairs = [d.con[i].pair for i in range(d.ncon) if PAIR_SELF0 <= d.con[i].pair < PAIR_BASE0]
        (hit if pairs else miss).append(arm)
    return hit[:n], miss[:n]


def test_self_collision_contacts_are_real_overlaps(model, oracle64):
    """Hull-hull self-collision (pairs 77..97): every MPR contact is between two polytopes that really
    intersect (an LP finds a common interior point of their H-representations), with the overlap along the
    normal at least the reported depth; arms whose hulls an LP proves disjoint get no such contact."""
    from scipy.optimize import linprog
    from gym_so100.model import PAIR_SELF0, PAIR_BASE0
    hit, miss = _self_configs(model, oracle64, 30, seed=8)

    def world(d, k):
        b = model.hull_body[k]
        R, p = np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])
        return _hull(model, k) @ R.T + p

    def depth_lp(V1, V2):
        """max t such that a point lies t inside both hulls (t < 0: separated)."""
        H1, H2 = ConvexHull(V1).equations, ConvexHull(V2).equations
        A = np.vstack([H1[:, :3], H2[:, :3]])
        b = -np.concatenate([H1[:, 3], H2[:, 3]])
        res = linprog(c=[0, 0, 0, -1], A_ub=np.hstack([A, np.ones((len(A), 1))]), b_ub=b,
                      bounds=[(None, None)] * 3 + [(None, 1.0)], method="highs")
        return -res.fun
    checked = 0
    for arm in hit:
        d = _state(oracle64, model, arm, (0.4, 0.95, 0.6, 1, 0, 0, 0))
        for i in range(d.ncon):
            p = d.con[i].pair
            if not PAIR_SELF0 <= p < PAIR_BASE0:
                continue
            k1, k2 = -1 - model.pair_geom1[p], -1 - model.pair_geom2[p]
            V1, V2 = world(d, k1), world(d, k2)
            assert depth_lp(V1, V2) > -1e-9, (p, depth_lp(V1, V2))
            n = np.array(d.con[i].frame[:3])
            assert (V1 @ n).max() - (V2 @ n).min() >= -d.con[i].dist - 1e-9
            checked += 1
    assert checked >= 30
    for arm in miss:
        d = _state(oracle64, model, arm, (0.4, 0.95, 0.6, 1, 0, 0, 0))
        for p in range(PAIR_SELF0, PAIR_BASE0):
            k1, k2 = -1 - model.pair_geom1[p], -1 - model.pair_geom2[p]
            if model.hull_body[k1] == model.hull_body[k2]:
                continue
            assert depth_lp(world(d, k1), world(d, k2)) < 1e-6, p


def test_base_contacts_are_real_overlaps(model, oracle64):
    """The static Base hull (pairs 98..106): every MPR contact of a link hull or the cube against it is
    between polytopes an LP shows to intersect, overlapping along the normal by at least the reported
    depth; arm poses whose link hulls the LP proves disjoint from the Base get no such contact.  The
    Base/Rotation_Pitch exclude (so_arm100.xml:165-167) leaves hull 0 out."""
    from scipy.optimize import linprog
    from gym_so100.model import PAIR_BASE0, PAIR_PADLINK0 as PAIR_PAD0, HULL_BASE   # the Base pairs end here
    rng = np.random.default_rng(21)
    lo = np.array([r[0] for r in model.jnt_range]); hi = np.array([r[1] for r in model.jnt_range])
    assert model.hull_body[HULL_BASE] == 1
    assert sorted(-1 - model.pair_geom2[p] for p in range(PAIR_BASE0 + 1, PAIR_PAD0)) == list(range(1, NHULL))

    def world(d, k):
        b = model.hull_body[k]
        R, p = np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])
        return _hull(model, k) @ R.T + p

    def depth_lp(V1, V2):
        H1, H2 = ConvexHull(V1).equations, ConvexHull(V2).equations
        A = np.vstack([H1[:, :3], H2[:, :3]])
        b = -np.concatenate([H1[:, 3], H2[:, 3]])
        res = linprog(c=[0, 0, 0, -1], A_ub=np.hstack([A, np.ones((len(A), 1))]), b_ub=b,
                      bounds=[(None, None)] * 3 + [(None, 1.0)], method="highs")
        return -res.fun
    checked = disjoint = 0
    for _ in range(120):
        d = _state(oracle64, model, rng.uniform(lo, hi), (0.4, 0.95, 0.6, 1, 0, 0, 0))
        if d.ncon_dropped:
            continue
        base = world(d, HULL_BASE)
        got = {d.con[i].pair: d.con[i] for i in range(d.ncon) if PAIR_BASE0 < d.con[i].pair < PAIR_PAD0}
        for p in range(PAIR_BASE0 + 1, PAIR_PAD0):
            V2 = world(d, -1 - model.pair_geom2[p])
            t = depth_lp(base, V2)
            if p in got:
                c = got[p]
                assert t > -1e-9, (p, t)
                n = np.array(c.frame[:3])
                assert (base @ n).max() - (V2 @ n).min() >= -c.dist - 1e-9
                checked += 1
            elif t < -1e-6:
                disjoint += 1
            else:
                assert t < 1e-6, (p, t)        # overlapping by more than the tolerance: a contact is due
    assert checked >= 10 and disjoint > 100
    # the cube pushed against the Base (pair 98): a contact exactly when the polytopes overlap
    hit = 0
    for _ in range(40):
        d0 = _state(oracle64, model, np.array(model.start_qpos[:]), (0.4, 0.95, 0.6, 1, 0, 0, 0))
        base = world(d0, HULL_BASE)
        q = rng.normal(size=4); q /= np.linalg.norm(q)
        c = base[rng.integers(len(base))] + rng.normal(0, 0.01, 3)
        d = _state(oracle64, model, np.array(model.start_qpos[:]), (*c, *q))
        if d.ncon_dropped:
            continue
        cube = _box_corners(c, _quat2mat(q), np.full(3, CUBE_HALF))
        t = depth_lp(cube, base)
        cons = [d.con[i] for i in range(d.ncon) if d.con[i].pair == PAIR_BASE0]
        if abs(t) < 1e-6:
            continue
        assert bool(cons) == (t > 0), (t, len(cons))
        hit += bool(cons)
    assert hit >= 5


def test_pad_link_contacts_are_real_overlaps(model, oracle64):
    """The finger pads against the arm's own link hulls (pairs 107..142, round 2: the last 36 of the 191
    pairs MuJoCo's filters leave): every MPR contact is between a pad box and a link hull that an LP shows
    to intersect, overlapping along the normal (pad -> hull) by at least the reported depth; pads an LP
    proves to overlap a link by more than the tolerance always get their contact.  Random arm poses fold the
    jaws onto the links."""
    from scipy.optimize import linprog
    from gym_so100.model import PAIR_PADLINK0, PAIR_MOCAPHULL0
    rng = np.random.default_rng(33)
    lo = np.array([r[0] for r in model.jnt_range]); hi = np.array([r[1] for r in model.jnt_range])
    assert PAIR_MOCAPHULL0 - PAIR_PADLINK0 == 36

    def world(d, k):
        b = model.hull_body[k]
        R, p = np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])
        return _hull(model, k) @ R.T + p

    def depth_lp(V1, V2):
        H1, H2 = ConvexHull(V1).equations, ConvexHull(V2).equations
        A = np.vstack([H1[:, :3], H2[:, :3]])
        b = -np.concatenate([H1[:, 3], H2[:, 3]])
        res = linprog(c=[0, 0, 0, -1], A_ub=np.hstack([A, np.ones((len(A), 1))]), b_ub=b,
                      bounds=[(None, None)] * 3 + [(None, 1.0)], method="highs")
        return -res.fun
    checked = overlaps = 0
    for _ in range(600):
        d = _state(oracle64, model, rng.uniform(lo, hi), (0.4, 0.95, 0.6, 1, 0, 0, 0))
        if d.ncon_dropped:
            continue
        got = {d.con[i].pair: d.con[i] for i in range(d.ncon) if PAIR_PADLINK0 <= d.con[i].pair < PAIR_MOCAPHULL0}
        for p in range(PAIR_PADLINK0, PAIR_MOCAPHULL0):
            g, k = model.pair_geom1[p], -1 - model.pair_geom2[p]
            R = np.array(d.geom_xmat[g][:]).reshape(3, 3)
            pad = _box_corners(np.array(d.geom_xpos[g][:]), R, np.array(model.geom_size[g][:]))
            link = world(d, k)
            lc = link.mean(0)
            if p not in got and (np.linalg.norm(pad.mean(0) - lc) > np.linalg.norm(pad - pad.mean(0), axis=1).max()
                                 + np.linalg.norm(link - lc, axis=1).max()):
                continue                           # bounding spheres apart: no overlap to miss
            t = depth_lp(pad, link)
            if p in got:
                c = got[p]
                assert t > -1e-9, (p, t)
                n = np.array(c.frame[:3])
                assert (pad @ n).max() - (link @ n).min() >= -c.dist - 1e-9
                checked += 1
            elif t > 1e-6:
                overlaps += 1                      # an overlap without its contact: must not happen
        if checked >= 30:
            break
    assert overlaps == 0
    assert checked >= 15, checked
