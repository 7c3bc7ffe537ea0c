"""Pin the oracle's task layer to the reference's own outputs (tests/golden/golden_task.npz).

The fixtures were produced by tests/golden/make_golden.py, which imports the reference's numpy code
(constants.py, utils.py, tasks/single_arm.py, env.py) in the build container.
"""
import numpy as np
import pytest

from gym_so100 import constants as C
from gym_so100 import utils as U

TASKS = (0, 1, 2)   # cube_to_bin, touch_cube, touch_cube_sparse (golden column order)


def test_unnormalize_bit_exact(golden, model, oracle64):
    for a, c in zip(golden["unnorm_action"], golden["unnorm_ctrl"]):
        got = oracle64.unnormalize(model, a)
        assert got.dtype == np.float32
        np.testing.assert_array_equal(got, c)


def test_unnormalize_host_mirror_matches_reference(golden):
    # the host-side numpy helper follows the same float32 write-back path (single_arm.py:33-38)
    for a, c in zip(golden["unnorm_action"], golden["unnorm_ctrl"]):
        x = a.copy()
        C.unnormalize_so100(x)
        np.testing.assert_array_equal(x, c)


def test_spawn_pose_bit_exact(golden, oracle64):
    for s, pose in zip(golden["spawn_seed"], golden["spawn_pose"]):
        np.testing.assert_array_equal(oracle64.spawn_pose(int(s)), pose)


def test_spawn_pose_host_mirror(golden):
    for s, pose in zip(golden["spawn_seed"][:64], golden["spawn_pose"][:64]):
        np.testing.assert_array_equal(U.sample_so100_box_pose(int(s)), pose)


@pytest.mark.parametrize("col,task", list(enumerate(TASKS)))
def test_reward_ladder(golden, model, oracle64, col, task):
    cube, ee, bits, want = golden["reward_cube"], golden["reward_ee"], golden["reward_bits"], golden["reward_value"]
    for i in range(len(cube)):
        got = oracle64.reward(model, task, cube[i].astype(np.float32), cube[i], ee[i], int(bits[i]))
        if task == 1:   # dense distance shaping: float arithmetic, compare to 1e-12
            assert abs(got - want[i, col]) <= 1e-12, (i, got, want[i, col])
        else:           # ladders: exact
            assert got == want[i, col], (i, got, want[i, col])


def test_reward_fixture_covers_every_rung(golden):
    rungs = set(np.unique(golden["reward_value"][:, 0]).tolist())
    assert {0.0, 1.0, 2.0, 2.5, 3.0, 4.0} <= rungs
    assert 4.0 in set(golden["reward_value"][:, 1]) and 4.0 in set(golden["reward_value"][:, 2])


def test_obs_packing_order(golden):
    # env.py:137-145: box, bin, ee, qpos[:6] as float32 (the inline comment at :71 is wrong)
    for x, obs in zip(golden["obs_in"], golden["obs_out"]):
        qpos, cube, ee = x[:13], x[13:16], x[16:19]
        bin_center = np.array([-0.2, 0.7, 0.001]) + np.array([0.0, 0.0, 0.02])
        want = np.concatenate([cube, bin_center, ee, qpos[:6]]).astype(np.float32)
        np.testing.assert_array_equal(obs.astype(np.float32), want)


def test_step_termination_semantics(golden):
    # env.py:175: terminated = is_success = reward == 4; truncated always False inside SO100Env
    for r, term, trunc, succ in golden["step_term"]:
        assert bool(term) == (r == 4.0) and bool(succ) == (r == 4.0) and not trunc


def test_goal_reward_reference(golden):
    a, d = golden["goal_achieved"], golden["goal_desired"]
    dist = np.linalg.norm(a - d, axis=1)
    np.testing.assert_array_equal(np.where(dist < 0.01, 0.0, -1.0).astype(np.float32), golden["goal_reward_batch"])
    np.testing.assert_array_equal(golden["goal_reward_single"], golden["goal_reward_batch"].astype(np.float64))
    np.testing.assert_array_equal(golden["goal_success"], dist < 0.01)
