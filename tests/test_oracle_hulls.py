"""Arm/jaw convex hulls vs the table top in the oracle: contact geometry against an
independent numpy evaluation of the model's hull data, condim-3 constraint rows, and the contacts
stopping an arm driven into the table (no MuJoCo here: the expected values are restated, not
MuJoCo's own)."""
import copy

import numpy as np

from gym_so100.model import NPAIR_BOX, NHULL, PAIR_MPR0, PAIR_PAD0

NV = 12


def _hulls(model):
    out = []
    for k in range(NHULL):
        s, n = model.hull_start[k], model.hull_count[k]
        v = np.array([[model.hull_vert[s + i][t] for t in range(3)] for i in range(n)])
        out.append((model.hull_body[k], v))
    return out


def _state(o, m, arm, box=(0.4, 0.95, 0.6, 1, 0, 0, 0)):
    d = o.new_data()
    o.reset(m, d, np.array(box, dtype=np.float64))
    for k in range(6):
        d.qpos[k] = arm[k]
    o.call("so100o_fwd_position", m, d)
    o.call("so100o_fwd_velocity", m, d)
    return d


def _expected(model, d, hulls):
    """(pair, pos, dist, fast) of every hull below the top.  fast: the top-face rule provably gives the exact minimum
    penetration (from the hull's body-frame bounding box: with D = top - its lowest point, an upper bound of the depth,
    the box's x-y extent lies inside the top face's footprint shrunk by D and the hull's centroid is at least D above
    the table's bottom): the contact is at the lowest vertex (first among ties), midway to the top.  Otherwise the pair
    goes through the convex collider (pos None: tests/test_oracle_epa.py grades it against the exact minimum
    penetration)."""
    top = model.table_top
    lo, hi = np.array(model.table_lo[:]), np.array(model.table_hi[:])
    bottom = top - 2 * model.geom_size[model.pair_geom1[NPAIR_BOX]][2]
    out = []
    for k, (b, v) in enumerate(hulls):
        R = np.array(d.xmat[b][:]).reshape(3, 3)
        P = np.array(d.xpos[b][:])
        c = R @ np.array(model.hull_center[k][:]) + P
        e = np.abs(R) @ np.array(model.hull_half[k][:])
        if not c[2] - e[2] < top:
            continue
        D = top - (c[2] - e[2])
        gz = (R @ np.array(model.hull_centroid[k][:]) + P)[2]
        fast = (c[0] - e[0] >= lo[0] + D and c[0] + e[0] <= hi[0] - D and c[1] - e[1] >= lo[1] + D and
                c[1] + e[1] <= hi[1] - D and gz - bottom >= D)
        w = v @ R.T + P
        i = int(np.argmin(w[:, 2]))
        if fast and w[i, 2] - top >= 0:
            continue                                 # the top-face rule: the lowest vertex above the top, separated
        pos = np.array([w[i, 0], w[i, 1], 0.5 * (w[i, 2] + top)]) if fast else None
        out.append((NPAIR_BOX + k, pos, w[i, 2] - top, fast))
    return out


def _dipping_configs(model, o, hulls, n, seed=0):
    rng = np.random.default_rng(seed)
    lo = np.array([r[0] for r in model.jnt_range]), np.array([r[1] for r in model.jnt_range])
    found = []
    while len(found) < n:
        arm = rng.uniform(lo[0], lo[1])
        d = _state(o, model, arm)
        if _expected(model, d, hulls):
            found.append(arm)
    return found


def test_hull_table_contacts_match_independent_geometry(model, oracle64):
    """The top-face rule's contacts (pairs 14..22) equal an independent numpy statement of it: one contact per hull
    below the top, at its lowest vertex, normal +z (table, geom1 -> hull, geom2), in hull order and ahead of the
    convex collider's contacts; hulls outside the rule's exact region (the table's edges and side faces) are in the
    list after the convex pairs 23..151 (tests/test_oracle_epa.py grades their depth against the exact minimum
    penetration)."""
    hulls = _hulls(model)
    assert sum(model.hull_count[k] for k in range(NHULL)) > 2000
    for arm in _dipping_configs(model, oracle64, hulls, 25):
        d = _state(oracle64, model, arm)
        want = _expected(model, d, hulls)
        pairs = [d.con[i].pair for i in range(d.ncon)]
        got = [(i, d.con[i].pair, np.array(d.con[i].pos[:]), d.con[i].dist, np.array(d.con[i].frame[:]))
               for i in range(d.ncon) if NPAIR_BOX <= d.con[i].pair < PAIR_MPR0]
        fast = [w for w in want if w[3]]
        assert [g[1] for g in got[:len(fast)]] == [w[0] for w in fast]      # hull order, one contact per hull
        for (i, p, pos, dist, fr), (_, wpos, wdist, _) in zip(got, fast):
            assert all(q < PAIR_MPR0 for q in pairs[:i])                       # ahead of the convex contacts
            np.testing.assert_allclose(pos, wpos, atol=1e-12)
            assert abs(dist - wdist) < 1e-12
            np.testing.assert_allclose(fr[:3], [0, 0, 1], atol=1e-15)  # table (geom1) -> hull (geom2)
            t1, t2 = fr[3:6], fr[6:9]
            assert abs(np.dot(t1, fr[:3])) < 1e-15 and abs(np.dot(t1, t2)) < 1e-15
        for i, p, _, _, _ in got[len(fast):]:                       # the collider's: after every convex pair
            assert p not in [w[0] for w in fast]
            assert all(q < PAIR_PAD0 for q in pairs[:i])
            assert not any(PAIR_MPR0 <= q < PAIR_PAD0 for q in pairs[i + 1:])


def test_hull_contacts_are_condim3_rows_on_arm_dofs(model, oracle64):
    hulls = _hulls(model)
    arm = _dipping_configs(model, oracle64, hulls, 1, seed=3)[0]
    d = _state(oracle64, model, arm)
    oracle64.call("so100o_fwd_acceleration", model, d)
    rows = [i for i in range(d.nefc) if d.efc_type[i] == 2 and d.efc_dim[i] > 0]
    hull_rows = [i for i in rows if NPAIR_BOX <= d.con[d.efc_id[i]].pair < PAIR_MPR0]
    assert hull_rows
    for i in hull_rows:
        assert d.efc_dim[i] == 3
        J = np.array([[d.efc_J[i + r][v] for v in range(NV)] for r in range(3)])
        assert np.abs(J[:, 6:]).max() == 0.0                  # the cube is not in the pair
        assert np.abs(J[:, :6]).max() > 0.0
        assert d.efc_force[i] >= 0.0                           # normal force (cone apex at 0)


def test_contacts_stop_the_arm_at_the_table(model, oracle64):
    """Drive the arm down into the table: with the hull contacts the lowest hull vertex stays within
    about a centimetre of the top (soft contacts, default solref 0.02, against the actuators' 3.5 N m),
    the finger pads' table contacts helping; with the table moved out of reach it sinks far below."""
    hulls = _hulls(model)
    no_table = copy.copy(model)
    no_table.table_top = -10.0
    no_table.geom_pos[0][2] -= 10.0          # the table geom too (the pads' box-box pairs, 98 + 6 i)

    def lowest(d):
        z = []
        for b, v in hulls:
            R = np.array(d.xmat[b][:]).reshape(3, 3)
            z.append((v @ R.T + np.array(d.xpos[b][:]))[:, 2].min())
        return min(z)

    # shoulder pitched forward, elbow and wrist folded down: the gripper is driven into the table
    target = np.array([0.0, 1.0, -1.0, 1.2, 0.0, 0.0])
    runs = {}
    for name, m in (("contacts", model), ("no_table", no_table)):
        d = _state(oracle64, m, np.array(model.start_qpos[:]))
        for k in range(6):
            d.ctrl[k] = target[k]
        zmin = 1.0
        for _ in range(600):
            oracle64.call("so100o_substep", m, d)
            zmin = min(zmin, lowest(d))
        runs[name] = zmin
    assert runs["no_table"] < -0.02, runs                      # the target really is below the table
    assert runs["contacts"] > -0.015, runs


def test_pad_contacts_match_independent_geometry(model, oracle64):
    """Finger pads vs the table (pairs 152..159): a box against the table mesh, the cube-table rule
    (the separating-axis minimum penetration over all 15 axes, one contact).  Over random arm poses a pad has one
    table contact exactly when it overlaps the table box; its depth is the exact minimum penetration (an independent
    scipy hull of the corner differences, within 1e-6) and along its normal the boxes overlap by that depth."""
    from gym_so100.model import PAIR_PAD0, PAIR_PADBIN0
    from test_oracle_epa import _exact, _points
    jlo = np.array([r[0] for r in model.jnt_range]); jhi = np.array([r[1] for r in model.jnt_range])
    rng = np.random.default_rng(4)
    touched = side = 0
    for _ in range(400):
        d = _state(oracle64, model, rng.uniform(jlo, jhi))
        assert d.ncon_dropped == 0
        got = {}
        for i in range(d.ncon):
            p = d.con[i].pair
            if PAIR_PAD0 <= p < PAIR_PADBIN0:
                got.setdefault(p, []).append(d.con[i])
        for pad in range(8):
            p = PAIR_PAD0 + pad
            A, B = _points(model, d, model.pair_geom1[p]), _points(model, d, 0)
            ex, _, _, _ = _exact(A, B)
            cons = got.get(p, [])
            if ex < -1e-9 or not cons:
                assert ex < 1e-9 and not cons, (pad, ex, len(cons))
                continue
            assert len(cons) == 1
            c = cons[0]
            n = np.array(c.frame[:3])
            # within 1e-6 (EPA's ccd_tolerance): the SAT pads |R| by 1e-6 (mjc_BoxBox's guard), 0.6 um on the table
            assert abs(-c.dist - ex) < 1e-6, (pad, -c.dist, ex)
            assert abs(((A @ n).max() - (B @ n).min()) - ex) < 1e-6      # pad (geom1) -> table (geom2)
            touched += 1
            side += n[2] > -0.99
    assert touched >= 20 and side >= 1, (touched, side)
