"""Device-side episode statistics (include/so100.h ep_return / ep_final / ep_accum; SURVEY §5 Metrics: the
reference trains under RecordEpisodeStatistics / SB3's Monitor, scripts/train_sac.py:290).  The kernel's
epilogue sums the float64 rewards in step order, so a host-side restatement of RecordEpisodeStatistics fed
the same float64 rewards and done flags must agree bit for bit, on the fused and the split step."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host_stats(venv, steps, rng):
    """Step venv `steps` times with random actions; return the host restatement's (final, accum, running)."""
    n = venv.num_envs
    ret = venv.ep_return.cpu().numpy().copy()
    length = venv.elapsed.cpu().numpy().astype(np.float64)
    final = venv.ep_final.cpu().numpy().copy()
    accum = venv.ep_accum.cpu().numpy().copy()
    ended = 0
    for _ in range(steps):
        a = torch.from_numpy(rng.uniform(-1, 1, (n, 6)).astype(np.float32)).to(venv.device)
        _, _, term, trunc, info = venv.step(a)
        r = venv.reward64.cpu().numpy()
        done = (term | trunc).cpu().numpy()
        succ = info["is_success"].cpu().numpy()
        ret = ret + r
        length = length + 1.0
        final[done, 0] = ret[done]
        final[done, 1] = length[done]
        accum[done, 0] += 1.0
        accum[done, 1] += succ[done].astype(np.float64)
        accum[done, 2] += ret[done]
        accum[done, 3] += length[done]
        ret[done] = 0.0
        length[done] = 0.0
        ended += int(done.sum())
        assert torch.equal(info["_episode"].cpu(), torch.from_numpy(done))
    return final, accum, ret, ended


@pytest.mark.parametrize("fused", [True, False])
def test_episode_statistics_match_host_restatement(fused):
    from gym_so100 import SO100VecEnv
    torch.cuda.set_device(0)
    n = 96
    v = SO100VecEnv(n, task="so100_touch_cube", device="cuda:0", seed=5, max_episode_steps=7, reward64=True,
                    episode_stats=True)
    v.fused = fused
    v.reset(seed=300)
    final, accum, ret, ended = _host_stats(v, 17, np.random.default_rng(1))
    torch.cuda.synchronize()
    assert ended >= 2 * n                                    # every env finished two 7-step episodes
    assert np.array_equal(v.ep_final.cpu().numpy(), final)
    assert np.array_equal(v.ep_accum.cpu().numpy(), accum)
    assert np.array_equal(v.ep_return.cpu().numpy(), ret)
    assert np.all((final[:, 1] >= 1.0) & (final[:, 1] <= 7.0))
    assert np.any(ret != 0.0)                                # the dense TouchCube shaping is non-zero
    s = v.episode_statistics(clear=True)
    assert s["episodes"] == int(accum[:, 0].sum()) and s["successes"] == int(accum[:, 1].sum())
    assert s["mean_length"] == pytest.approx(accum[:, 3].sum() / accum[:, 0].sum(), rel=1e-12)
    assert s["mean_return"] == pytest.approx(accum[:, 2].sum() / accum[:, 0].sum(), rel=1e-12)
    assert float(v.ep_accum.abs().sum()) == 0.0
    # a reset (here of every other env) starts the running return again
    mask = torch.arange(n, device=v.device) % 2 == 0
    v.reset(mask=mask)
    r = v.ep_return.cpu().numpy()
    assert np.all(r[0::2] == 0.0) and np.array_equal(r[1::2], ret[1::2])
    v.close()


@pytest.mark.parametrize("fused", [True, False])
def test_episode_statistics_without_autoreset(fused):
    """autoreset=False and no reset after the TimeLimit: the env keeps reporting truncated, but its episode is
    counted once, with its length at the limit (the totals grew on every later step before)."""
    from gym_so100 import SO100VecEnv
    torch.cuda.set_device(0)
    n = 32
    v = SO100VecEnv(n, device="cuda:0", seed=5, max_episode_steps=5, reward64=True, episode_stats=True,
                    autoreset=False)
    v.fused = fused
    v.reset(seed=40)
    a = torch.zeros(n, 6, device=v.device)
    for t in range(9):
        _, _, term, trunc, _ = v.step(a)
        torch.cuda.synchronize()
        assert bool(trunc.all()) == (t >= 4)
    acc = v.ep_accum.cpu().numpy()
    assert not term.any()
    assert np.all(acc[:, 0] == 1.0) and np.all(acc[:, 3] == 5.0)
    assert np.all(v.ep_final.cpu().numpy()[:, 1] == 5.0)
    v.close()


def test_sb3_episode_info():
    """VecMonitor's info["episode"] for the envs that finished, from the kernel's statistics."""
    from gym_so100.sb3 import SO100SB3VecEnv
    torch.cuda.set_device(0)
    n = 16
    env = SO100SB3VecEnv(n, task="so100_touch_cube", device="cuda:0", seed=2, max_episode_steps=5)
    env.seed(11)
    env.reset()
    rng = np.random.default_rng(0)
    total = np.zeros(n)
    for t in range(5):
        obs, rew, dones, infos = env.step(rng.uniform(-1, 1, (n, 6)).astype(np.float32))
        total += env.venv.reward64.cpu().numpy() if env.venv.reward64 is not None else rew
        if t < 4:
            assert not dones.any() and all("episode" not in i for i in infos)
    assert dones.all()
    for i in range(n):
        ep = infos[i]["episode"]
        assert ep["l"] == 5 and ep["t"] >= 0.0
        assert ep["r"] == pytest.approx(total[i], rel=1e-6, abs=1e-6)
    env.close()
