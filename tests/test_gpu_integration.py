"""The reference-side ctypes binding of INTEGRATION.md §2, executed: a single-env adapter built only on
the C-ABI (no SO100VecEnv) must reproduce SO100VecEnv's reset / step outputs bit-for-bit."""
import ctypes

import numpy as np
import pytest
import torch

from gym_so100 import _native
from gym_so100.model import build_model

pytestmark = pytest.mark.gpu

_TASK = {"so100_cube_to_bin": 0, "so100_touch_cube": 1, "so100_touch_cube_sparse": 2}


class HipPhysicsBackend:
    """Copy of INTEGRATION.md §2 (imports adapted to this repo's package name)."""

    def __init__(self, task, device="cuda:0"):
        self.lib = _native.load()
        self.model = build_model()
        self.dev = torch.device(device)
        self.h = self.lib.so100_create(ctypes.byref(self.model), 1, self.dev.index or 0)
        if not self.h:
            raise RuntimeError(self.lib.so100_last_error().decode())
        _native.check(self.lib.so100_configure(self.h, _TASK[task], 0, ctypes.c_uint64(0), 0), "configure")
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=self.dev)
        self.t = dict(qpos=z(1, 13), qvel=z(1, 12), qacc_warmstart=z(1, 12), elapsed=z(1, dt=torch.int32),
                      episode=z(1, dt=torch.int32), action=z(1, 6), obs=z(1, 15), reward=z(1),
                      terminated=z(1, dt=torch.bool), truncated=z(1, dt=torch.bool),
                      success=z(1, dt=torch.bool), contact_bits=z(1, dt=torch.int32))
        self.b = _native.SO100Buffers()
        for k, v in self.t.items():
            setattr(self.b, k, v.data_ptr())
        self.seed_t = z(1, dt=torch.int32)                          # uint32 seeds, stored as int32 bits

    def reset(self, seed=None):
        seeds = None
        if seed is not None:
            s = int(seed)
            if not 0 <= s < 2 ** 32:
                raise ValueError("Seed must be between 0 and 2**32 - 1")
            self.seed_t.fill_(int(np.array(s, np.uint32).view(np.int32)))
            seeds = ctypes.c_void_p(self.seed_t.data_ptr())
        _native.check(self.lib.so100_reset(self.h, ctypes.byref(self.b), None, seeds, None), "so100_reset")
        return self.t["obs"][0].cpu().numpy()

    def step(self, action):
        self.t["action"].copy_(torch.as_tensor(np.asarray(action, np.float32)).view(1, 6))
        _native.check(self.lib.so100_step(self.h, ctypes.byref(self.b), 0, None), "so100_step")
        obs = self.t["obs"][0].cpu().numpy()
        reward = float(self.t["reward"][0])
        return obs, reward, reward == 4

    def close(self):
        self.lib.so100_destroy(self.h)


def test_reference_side_binding_matches_vec_env():
    from gym_so100 import SO100VecEnv
    torch.cuda.set_device(0)
    be = HipPhysicsBackend("so100_cube_to_bin")
    ve = SO100VecEnv(1, task="so100_cube_to_bin", device="cuda:0", autoreset=False, max_episode_steps=0)
    o1 = be.reset(1234)
    o2, _ = ve.reset(seed=1234)
    np.testing.assert_array_equal(o1, o2[0].cpu().numpy())
    rng = np.random.default_rng(0)
    for _ in range(20):
        a = rng.uniform(-1, 1, 6).astype(np.float32)
        ob1, r1, t1 = be.step(a)
        ob2, r2, t2, _, _ = ve.step(torch.from_numpy(a).view(1, 6).cuda())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ob1, ob2[0].cpu().numpy())
        assert r1 == float(r2[0]) and t1 == bool(t2[0])
    # seeds >= 2**31 spawn as RandomState(seed) does (no sign-bit mask), seed=None resets with a fresh spawn
    for seed in (2 ** 31 + 12345, 2 ** 32 - 1):
        o1 = be.reset(seed)
        o2, _ = ve.reset(seed=[seed])
        np.testing.assert_array_equal(o1, o2[0].cpu().numpy())
        pose = ve.spawn_pose([seed]).cpu().numpy()[0]                # device MT19937 == RandomState(seed)
        np.testing.assert_array_equal(ve.qpos[0, 6:9].cpu().numpy(), pose[:3].astype(np.float32))
        np.testing.assert_array_equal(pose, np.random.RandomState(seed).uniform([-0.25, 0.3, 0.05], [-0.15, 0.6, 0.05])
                                      .tolist() + [1.0, 0.0, 0.0, 0.0])
    o3 = be.reset(None)
    assert np.all(np.isfinite(o3))
    with pytest.raises(ValueError):
        be.reset(2 ** 32)
    be.close()
    ve.close()
