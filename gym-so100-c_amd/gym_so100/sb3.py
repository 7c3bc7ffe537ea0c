"""stable-baselines3 VecEnv adapter over SO100VecEnv.

The reference's training scripts drive gym_so100 through SB3: ``make_vec_env(..., SubprocVecEnv)`` +
``VecNormalize`` (reference scripts/train_sac.py:294-310) and ``DummyVecEnv`` + ``HerReplayBuffer``
for the GoalEnv (scripts/train_sac_her.py:231-251).  ``SO100SB3VecEnv`` is a drop-in for those
vectorised envs: one object stepping N envs on the GPU with SB3's VecEnv contract:

* ``reset() -> obs`` (numpy, or a dict of numpy arrays for the GoalEnv), seeded by ``seed(s)`` as
  SB3 does (env i <- s + i, one-shot);
* ``step_async(actions)`` / ``step_wait() -> (obs, rewards, dones, infos)`` with ``dones = terminated
  | truncated`` and SB3's auto-reset conventions per done env: ``infos[i]["terminal_observation"]``
  (the finished episode's last observation) and ``infos[i]["TimeLimit.truncated"]`` (truncated and not
  terminated); every info carries ``is_success``;
* ``env_method("compute_reward", achieved, desired, infos)`` for HER (batched, on the device);
* ``get_attr`` / ``set_attr`` / ``env_is_wrapped`` / ``seed`` / ``close`` / ``get_images``.

When stable-baselines3 is importable the class derives from its ``VecEnv`` (so ``VecNormalize`` and
``isinstance`` checks accept it); otherwise it is a duck-typed equivalent.  The physics stays on the
GPU; this layer only moves the [N,15] observation and the per-env scalars to host numpy, which SB3's
numpy interface requires.
"""
import time

import numpy as np

from . import spaces
from .vec_env import SO100VecEnv

try:  # optional dependency (absent in this image)
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except ImportError:  # pragma: no cover - exercised when SB3 is installed
    _VecEnvBase = object


def _np(t):
    return t.detach().cpu().numpy()


class SO100SB3VecEnv(_VecEnvBase):
    """N SO-ARM100 envs on one GPU behind SB3's VecEnv interface (numpy in / numpy out)."""

    metadata = {"render_modes": []}

    def __init__(self, num_envs, task="so100_cube_to_bin", device="cuda:0", seed=0, max_episode_steps=None,
                 domain_randomization=None, env_offset=0, iterations=None, solver="newton"):
        self.venv = SO100VecEnv(num_envs, task=task, device=device, seed=seed, max_episode_steps=max_episode_steps,
                                autoreset=True, domain_randomization=domain_randomization, env_offset=env_offset,
                                iterations=iterations, solver=solver, episode_stats=True)
        self._t0 = time.time()
        n = self.venv.num_envs
        obs_box = spaces.Box(low=-np.inf, high=np.inf, shape=(15,), dtype=np.float32)
        if self.venv.is_goal:
            obs_space = spaces.Dict({
                "observation": obs_box,
                "achieved_goal": spaces.Box(low=-np.inf, high=np.inf, shape=(3,), dtype=np.float32),
                "desired_goal": spaces.Box(low=-np.inf, high=np.inf, shape=(3,), dtype=np.float32)})
        else:
            obs_space = obs_box
        act_space = spaces.Box(low=-1, high=1, shape=(6,), dtype=np.float32)
        if _VecEnvBase is not object:
            super().__init__(n, obs_space, act_space)
        else:
            self.num_envs = n
            self.observation_space = obs_space
            self.action_space = act_space
            self.render_mode = None
        self._next_seeds = None
        self._actions = None
        self.reset_infos = [{} for _ in range(n)]

    # ------------------------------------------------------------------ SB3 VecEnv API
    def seed(self, seed=None):
        """Seeds for the next reset(): env i <- seed + i (SB3 VecEnv.seed); None -> in-kernel seeds."""
        if seed is None:
            self._next_seeds = None
            return [None] * self.num_envs
        self._next_seeds = int(seed)
        return [int(seed) + i for i in range(self.num_envs)]

    def reset(self):
        seed, self._next_seeds = self._next_seeds, None
        obs, _ = self.venv.reset(seed=seed)
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return self._obs_np(obs)

    def step_async(self, actions):
        a = np.asarray(actions, dtype=np.float32)
        if a.shape != (self.num_envs, 6):
            raise ValueError(f"actions must be [{self.num_envs}, 6], got {a.shape}")
        self._actions = a

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        v = self.venv
        prev_goal = v.desired_goal.clone() if v.is_goal else None   # the auto-reset resamples done envs' goals
        obs, rew, term, trunc, info = v.step(self._actions)
        self._actions = None
        done_t = term | trunc
        rewards = _np(rew).astype(np.float32)
        terminated, truncated = _np(term), _np(trunc)
        dones = terminated | truncated
        success = _np(info["is_success"])
        infos = [{"is_success": bool(success[i])} for i in range(self.num_envs)]
        idx = np.flatnonzero(dones)
        if idx.size:
            final = _np(v.final_obs[done_t])
            if v.is_goal:
                fgoal = _np(prev_goal[done_t])
            for k, i in enumerate(idx):
                if v.is_goal:
                    term_obs = {"observation": final[k], "achieved_goal": final[k, 0:3].copy(),
                                "desired_goal": fgoal[k]}
                else:
                    term_obs = final[k]
                infos[i]["terminal_observation"] = term_obs
                infos[i]["TimeLimit.truncated"] = bool(truncated[i] and not terminated[i])
            # VecMonitor's info["episode"], from the kernel's episode statistics (return in float64, as the
            # reference's rewards)
            ep = _np(v.ep_final[done_t])
            t = round(time.time() - self._t0, 6)
            for k, i in enumerate(idx):
                infos[i]["episode"] = {"r": float(ep[k, 0]), "l": int(ep[k, 1]), "t": t}
        return self._obs_np(obs), rewards, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def get_images(self):
        return [None] * self.num_envs      # camera renders are out of scope

    def render(self, mode=None):
        return None

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, (int, np.integer)):
            return [int(indices)]
        return [int(i) for i in indices]

    def get_attr(self, attr_name, indices=None):
        val = getattr(self.venv, attr_name) if hasattr(self.venv, attr_name) else getattr(self, attr_name)
        return [val for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        if hasattr(self.venv, attr_name):
            raise AttributeError(f"{attr_name!r} is shared by all envs of the batch and cannot be set per env")
        setattr(self, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = self._indices(indices)
        if method_name == "compute_reward":
            # HerReplayBuffer: one batched call for the first index, answered on the device
            achieved, desired = method_args[0], method_args[1]
            r = _np(self.venv.compute_reward(achieved, desired))
            shape = np.shape(achieved)[:-1]
            return [r.reshape(shape)] + [None] * (len(idx) - 1)
        fn = getattr(self.venv, method_name)
        out = fn(*method_args, **method_kwargs)
        return [out for _ in idx]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    # ------------------------------------------------------------------ helpers
    def _obs_np(self, obs):
        if isinstance(obs, dict):
            return {k: _np(t) for k, t in obs.items()}
        return _np(obs)

    @property
    def unwrapped(self):
        return self

    @property
    def device(self):
        return self.venv.device
