"""SB3 VecEnv adapter (gym_so100/sb3.py) on the GPU: SB3's auto-reset contract
(terminal_observation, TimeLimit.truncated, is_success), seed() semantics and HER's compute_reward."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def test_sb3_reset_seed_and_terminal_observation():
    from gym_so100 import SO100VecEnv
    from gym_so100.sb3 import SO100SB3VecEnv
    n, limit = 48, 5
    env = SO100SB3VecEnv(n, seed=3, max_episode_steps=limit)
    ref = SO100VecEnv(n, seed=3, max_episode_steps=0, autoreset=False)     # same episodes, never reset
    assert env.seed(7) == [7 + i for i in range(n)]
    obs = env.reset()
    ref_obs, _ = ref.reset(seed=7)
    assert isinstance(obs, np.ndarray) and obs.shape == (n, 15) and obs.dtype == np.float32
    np.testing.assert_array_equal(obs, ref_obs.cpu().numpy())
    # cube spawn = RandomState(7 + i) (utils.py:18-29): obs[0:3] is the cube site, a fixed body-frame
    # offset from the spawned body origin (identity orientation at reset)
    spawn = env.venv.spawn_pose(np.arange(7, 7 + n)).cpu().numpy()
    off = obs[:, 0:2] - spawn[:, 0:2]
    np.testing.assert_allclose(off, np.repeat(off[:1], n, 0), atol=1e-6)
    rng = np.random.default_rng(0)
    for t in range(limit):
        a = rng.uniform(-1, 1, size=(n, 6)).astype(np.float32)
        obs, rew, dones, infos = env.step(a)
        r_obs, r_rew, r_term, _, _ = ref.step(torch.from_numpy(a))
        r_obs, r_term = r_obs.cpu().numpy(), r_term.cpu().numpy()
        assert rew.dtype == np.float32 and dones.dtype == np.bool_ and len(infos) == n
        np.testing.assert_array_equal(rew, r_rew.cpu().numpy())
        for i in range(n):
            assert "is_success" in infos[i]
            if dones[i]:
                np.testing.assert_array_equal(infos[i]["terminal_observation"], r_obs[i])
                assert infos[i]["TimeLimit.truncated"] == (t == limit - 1 and not r_term[i])
        if t < limit - 1:
            live = ~dones
            np.testing.assert_array_equal(obs[live], r_obs[live])
    assert dones.all()                                   # TimeLimit: every episode ended at step `limit`
    # the returned obs are fresh episodes: arm back at the start pose
    np.testing.assert_allclose(obs[:, 9:15], np.repeat(obs[:1, 9:15], n, 0), atol=1e-6)
    assert env.env_is_wrapped(object) == [False] * n
    assert env.get_attr("num_envs", [0, 1]) == [n, n]
    env.close()
    ref.close()


def test_sb3_goal_env_her_contract():
    from gym_so100.sb3 import SO100SB3VecEnv
    n = 16
    env = SO100SB3VecEnv(n, task="so100_goal", seed=5, max_episode_steps=3)
    obs = env.reset()
    assert set(obs) == {"observation", "achieved_goal", "desired_goal"}
    assert obs["observation"].shape == (n, 15) and obs["desired_goal"].shape == (n, 3)
    np.testing.assert_array_equal(obs["achieved_goal"], obs["observation"][:, 0:3])
    # HER relabelling: batched compute_reward through env_method (env.py:341-353)
    ach = obs["achieved_goal"]
    r = env.env_method("compute_reward", ach, obs["desired_goal"], [{}] * n, indices=[0])[0]
    d = np.linalg.norm(ach - obs["desired_goal"], axis=-1)
    np.testing.assert_array_equal(r, np.where(d < 0.01, 0.0, -1.0).astype(np.float32))
    assert np.all(env.env_method("compute_reward", ach, ach, [{}] * n, indices=[0])[0] == 0.0)
    goals = obs["desired_goal"].copy()
    for t in range(3):
        obs, rew, dones, infos = env.step(np.zeros((n, 6), np.float32))
    assert dones.all()
    for i in range(n):
        term = infos[i]["terminal_observation"]
        np.testing.assert_array_equal(term["desired_goal"], goals[i])       # the finished episode's goal
        np.testing.assert_array_equal(term["achieved_goal"], term["observation"][0:3])
    env.close()
