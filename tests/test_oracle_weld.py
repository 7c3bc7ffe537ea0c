"""EE / mocap variant: the weld equality of so_arm100_ee.xml:171-173 in the oracle.

MuJoCo is absent, so the restatement of mj_makeEquality's weld rows is pinned by properties its
derivation fixes: the Jacobian rows are the derivative of the residual (finite differences), the
exact elimination of the always-active rows into (M, qfrc) reproduces the unreduced quadratic, and the
constraint pulls the end effector to the mocap target.  Parity with MuJoCo itself is unpinned."""
import numpy as np
import pytest

from gym_so100.model import build_model

NV = 12


@pytest.fixture(scope="module")
def models():
    return {v: build_model(solver="newton", variant=v) for v in ("joint", "ee")}


def state(o, m, arm, mocap_pos, mocap_quat, qvel=None, box=(-0.2, 0.45, 0.3, 1, 0, 0, 0)):
    d = o.new_data()
    o.reset(m, d, np.array(box, np.float64))
    for k in range(6):
        d.qpos[k] = float(arm[k])
    if qvel is not None:
        for k in range(NV):
            d.qvel[k] = float(qvel[k])
    for k in range(3):
        d.mocap_pos[k] = float(mocap_pos[k])
    for k in range(4):
        d.mocap_quat[k] = float(mocap_quat[k])
    o.call("so100o_fwd_position", m, d)
    o.call("so100o_fwd_velocity", m, d)
    return d


def ee_frame(d):
    return np.array(d.xpos[6][:]), np.array(d.xmat[6][:]).reshape(3, 3)


def rand_quat(rng, scale):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = rng.uniform(-scale, scale)
    return np.r_[np.cos(a / 2), np.sin(a / 2) * ax]


def test_weld_jacobian_is_residual_derivative(models, oracle64):
    m = models["ee"]
    rng = np.random.default_rng(0)
    for _ in range(10):
        arm = rng.uniform(-1.0, 1.0, 6)
        mp, mq = rng.uniform([-0.3, 0.3, 0.05], [0.0, 0.6, 0.3]), rand_quat(rng, 2.5)
        d = state(oracle64, m, arm, mp, mq)
        J = np.array([d.weld_J[i][:] for i in range(6)])
        r0 = np.array(d.weld_pos[:])
        eps = 1e-6
        for j in range(6):
            a2 = arm.copy()
            a2[j] += eps
            dp = state(oracle64, m, a2, mp, mq)
            a3 = arm.copy()
            a3[j] -= eps
            dm = state(oracle64, m, a3, mp, mq)
            fd = (np.array(dp.weld_pos[:]) - np.array(dm.weld_pos[:])) / (2 * eps)
            np.testing.assert_allclose(J[:, j], fd, atol=2e-6, rtol=1e-5)
        assert np.all(J[:, 5] == 0)                        # the Jaw hinge is not on the ee chain
        assert np.linalg.norm(r0[3:]) <= 1.0               # imag part of a w >= 0 unit quaternion


def test_weld_elimination_is_exact(models, oracle64):
    """M' = M + J'DJ and M' a0' = M a0 + J'D aref: the reduced Gauss cost equals Gauss + weld cost up to a
    constant, so both problems have the same minimiser."""
    rng = np.random.default_rng(1)
    for _ in range(10):
        arm = rng.uniform(-1.0, 1.0, 6)
        qvel = rng.normal(0, 0.5, NV)
        mp, mq = rng.uniform([-0.3, 0.3, 0.05], [0.0, 0.6, 0.3]), rand_quat(rng, 2.5)
        d0 = state(oracle64, models["joint"], arm, mp, mq, qvel)
        d1 = state(oracle64, models["ee"], arm, mp, mq, qvel)
        for d in (d0, d1):
            oracle64.call("so100o_fwd_acceleration", models["ee"] if d is d1 else models["joint"], d)
        M0 = np.array([d0.qM[i][:] for i in range(NV)])
        M1 = np.array([d1.qM[i][:] for i in range(NV)])
        J = np.array([d1.weld_J[i][:] for i in range(6)])
        D = np.array(d1.weld_D[:])
        aref = np.array(d1.weld_aref[:])
        np.testing.assert_allclose(M1, M0 + J.T @ np.diag(D) @ J, rtol=1e-12, atol=1e-12 * np.abs(M1).max())
        a0, a1 = np.array(d0.qacc_smooth[:]), np.array(d1.qacc_smooth[:])
        lhs, rhs = M1 @ a1, M0 @ a0 + J.T @ (D * aref)
        np.testing.assert_allclose(lhs, rhs, rtol=1e-9, atol=1e-9 * np.abs(rhs).max())
        # cost identity at random accelerations
        c = None
        for _ in range(3):
            a = rng.normal(0, 5, NV)
            full = 0.5 * (a - a0) @ M0 @ (a - a0) + 0.5 * np.sum(D * (J @ a - aref) ** 2)
            red = 0.5 * (a - a1) @ M1 @ (a - a1)
            c = full - red if c is None else c
            assert abs((full - red) - c) <= 1e-8 * max(1.0, abs(full))


def test_weld_pulls_ee_to_target(models, oracle64):
    """Mocap target 3 cm from the end effector: the weld closes the gap (position and orientation).  The marker box
    at the target (so_arm100_ee.xml:155) collides with the gripper's links (test_marker_box_blocks_the_gripper), so
    this weld-only property is checked with the box shrunk to a point."""
    from gym_so100.model import MOCAP_GEOM, build_model
    m = build_model(solver="newton", variant="ee")
    for k in range(3):
        m.geom_size[MOCAP_GEOM][k] = 1e-5
    d = state(oracle64, m, np.zeros(6), np.zeros(3), np.array([1.0, 0, 0, 0]))
    p0 = np.array(d.site_ee[:])
    _, R = ee_frame(d)
    # current ee_site frame as the target, then displaced
    from scipy.spatial.transform import Rotation
    q = Rotation.from_matrix(R).as_quat()[[3, 0, 1, 2]]
    target = p0 + np.array([0.0, 0.03, 0.0])
    d = state(oracle64, m, np.zeros(6), target, q)
    dist0 = np.linalg.norm(np.array(d.site_ee[:]) - target)
    act = np.zeros(6, np.float32)
    for _ in range(60):
        oracle64.env_step(m, d, 0, act)
    dist = np.linalg.norm(np.array(d.site_ee[:]) - target)
    assert dist0 > 0.029 and dist < 0.5 * dist0, (dist0, dist)
    assert np.linalg.norm(np.array(d.weld_pos[3:])) < 0.05        # orientation held


def test_marker_box_blocks_the_gripper(models, oracle64):
    """The EE variant's mocap marker (a 4 x 12 x 4 cm box, default contype/conaffinity) is a collision geom in MuJoCo:
    centred on a target 3 cm from the end effector it overlaps the wrist and jaw link hulls (pairs 143..151), and
    its contacts hold the gripper off where the weld alone would pull it in (test_weld_pulls_ee_to_target)."""
    from gym_so100.model import PAIR_MOCAPHULL0, PAIR_PAD0
    m = models["ee"]
    d = state(oracle64, m, np.zeros(6), np.zeros(3), np.array([1.0, 0, 0, 0]))
    p0 = np.array(d.site_ee[:])
    _, R = ee_frame(d)
    from scipy.spatial.transform import Rotation
    q = Rotation.from_matrix(R).as_quat()[[3, 0, 1, 2]]
    target = p0 + np.array([0.0, 0.03, 0.0])
    d = state(oracle64, m, np.zeros(6), target, q)
    marker = [d.con[i].pair for i in range(d.ncon) if PAIR_MOCAPHULL0 <= d.con[i].pair < PAIR_PAD0]
    assert len(marker) >= 2, marker
    dist0 = np.linalg.norm(np.array(d.site_ee[:]) - target)
    act = np.zeros(6, np.float32)
    for _ in range(60):
        oracle64.env_step(m, d, 0, act)
    dist = np.linalg.norm(np.array(d.site_ee[:]) - target)
    assert dist > 0.8 * dist0, (dist0, dist)
    # the joint variant has no marker: none of its pairs ever appears there
    mj = models["joint"]
    dj = state(oracle64, mj, np.zeros(6), target, q)
    assert not any(PAIR_MOCAPHULL0 <= dj.con[i].pair < PAIR_PAD0 or dj.con[i].pair >= PAIR_PAD0 + 48
                   for i in range(dj.ncon))
