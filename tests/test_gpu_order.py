"""The fused step's heavy-first wave order (so100_step.hip so100_order_kernel): from 1,028 envs up
(more than 256 four-env groups) every launch takes its groups in the order the order kernel wrote from the previous
step's per-group costs, one workgroup per XCD range since round 6.  The order must be a permutation of the groups: a
group left out would not be stepped and one listed twice would be stepped twice.  Checked through the step counter,
which every stepped env advances by one, and bitwise against the same envs stepped in the split path (no order)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [8192, 65536 + 4 * 37 + 1])
def test_order_steps_every_env_once(n):
    from gym_so100 import SO100VecEnv
    env = SO100VecEnv(n, device="cuda:0", seed=0, autoreset=False, max_episode_steps=0)
    env.reset(seed=7)
    g = torch.Generator(device="cuda").manual_seed(0)
    e0 = env.elapsed.clone()
    for _ in range(4):
        env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    assert env.fused
    assert torch.equal(env.elapsed - e0, torch.full_like(e0, 4)), "an env was stepped other than once per step"
    assert bool(torch.isfinite(env.qpos).all())


def test_order_bitwise_against_split():
    """4,096 envs (1,024 groups: ordered) in the fused step, the same envs in the split path: equal bit for bit."""
    from gym_so100 import SO100VecEnv
    n = 4096
    out = []
    for fused in (True, False):
        env = SO100VecEnv(n, device="cuda:0", seed=0, autoreset=False, max_episode_steps=0)
        env.fused = fused
        env.reset(seed=11)
        g = torch.Generator(device="cuda").manual_seed(1)
        for _ in range(3):
            env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
        torch.cuda.synchronize()
        out.append((env.qpos.cpu().numpy().copy(), env.qvel.cpu().numpy().copy()))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
