"""Arm/jaw convex hulls vs the table top in the oracle: contact geometry against an
independent numpy evaluation of the model's hull data, condim-3 constraint rows, and the contacts
stopping an arm driven into the table (no MuJoCo here: the expected values are restated, not
MuJoCo's own)."""
import copy

import numpy as np

from gym_so100.model import NPAIR_BOX, NHULL, PAIR_MPR0

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
    """(pair, pos, dist) of every hull below the top: lowest in-footprint vertex, first among ties."""
    top = model.table_top
    lo, hi = np.array(model.table_lo[:]), np.array(model.table_hi[:])
    out = []
    for k, (b, v) in enumerate(hulls):
        R = np.array(d.xmat[b][:]).reshape(3, 3)
        w = v @ R.T + np.array(d.xpos[b][:])
        inside = (w[:, 0] >= lo[0]) & (w[:, 0] <= hi[0]) & (w[:, 1] >= lo[1]) & (w[:, 1] <= hi[1])
        if not inside.any():
            continue
        i = np.flatnonzero(inside)[np.argmin(w[inside, 2])]
        if w[i, 2] - top < 0:
            out.append((NPAIR_BOX + k, np.array([w[i, 0], w[i, 1], 0.5 * (w[i, 2] + top)]), w[i, 2] - top))
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
    hulls = _hulls(model)
    assert sum(model.hull_count[k] for k in range(NHULL)) > 2000
    for arm in _dipping_configs(model, oracle64, hulls, 25):
        d = _state(oracle64, model, arm)
        want = _expected(model, d, hulls)
        got = [(d.con[i].pair, np.array(d.con[i].pos[:]), d.con[i].dist, np.array(d.con[i].frame[:]))
               for i in range(d.ncon) if NPAIR_BOX <= d.con[i].pair < PAIR_MPR0]
        assert [g[0] for g in got] == [w[0] for w in want]          # hull order, one contact per hull
        for (p, pos, dist, fr), (_, wpos, wdist) in zip(got, want):
            np.testing.assert_allclose(pos, wpos, atol=1e-12)
            assert abs(dist - wdist) < 1e-12
            np.testing.assert_allclose(fr[:3], [0, 0, 1], atol=1e-15)  # table (geom1) -> hull (geom2)
            t1, t2 = fr[3:6], fr[6:9]
            assert abs(np.dot(t1, fr[:3])) < 1e-15 and abs(np.dot(t1, t2)) < 1e-15


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
    """Finger pads vs the table (pairs 98..105), against an independent numpy statement of
    the rule: over random arm poses, a pad gets one table contact exactly when one of its 8 corners lies
    inside the top face's footprint and below the top; distance = the deepest such corner's height, x-y =
    those corners' centroid, z midway between the deepest corner and the top, normal from the pad
    (geom1) down into the table."""
    from gym_so100.model import PAIR_PAD0, PAIR_PADBIN0
    top = model.table_top
    lo, hi = np.array(model.table_lo[:]), np.array(model.table_hi[:])
    jlo = np.array([r[0] for r in model.jnt_range]); jhi = np.array([r[1] for r in model.jnt_range])
    rng = np.random.default_rng(4)
    signs = np.array([[1 if k & 1 else -1, 1 if k & 2 else -1, 1 if k & 4 else -1] for k in range(8)], float)
    touched = 0
    for _ in range(400):
        d = _state(oracle64, model, rng.uniform(jlo, jhi))
        if d.ncon_dropped:
            continue                         # contact set truncated at SO100_MAXCON: not this test's subject
        got = {}
        for i in range(d.ncon):
            p = d.con[i].pair
            if PAIR_PAD0 <= p < PAIR_PADBIN0:
                got.setdefault(p, []).append(d.con[i])
        for pad in range(8):
            g = model.pair_geom1[PAIR_PAD0 + pad]
            R = np.array(d.geom_xmat[g][:]).reshape(3, 3)
            w = (signs * np.array(model.geom_size[g][:])) @ R.T + np.array(d.geom_xpos[g][:])
            sel = ((w[:, :2] >= lo) & (w[:, :2] <= hi)).all(1) & (w[:, 2] < top)
            cons = got.get(PAIR_PAD0 + pad, [])
            assert len(cons) == int(sel.any()), (pad, len(cons), sel)
            if not cons:
                continue
            touched += 1
            c, zmin = cons[0], w[sel, 2].min()
            np.testing.assert_allclose(c.frame[:3], [0, 0, -1], atol=0)
            assert abs(c.dist - (zmin - top)) < 1e-12
            np.testing.assert_allclose(c.pos[:], [*w[sel, :2].mean(0), 0.5 * (zmin + top)], atol=1e-12)
    assert touched >= 20
