"""``make(id, **kwargs)``: the reference's ``gym.make`` for its registered ids, without gymnasium.

The reference registers three ids (gym_so100/__init__.py:4-32) whose entry point is ``SO100Env`` with
``obs_type="so100_pixels_agent_pos"`` and a TimeLimit of 300 (TouchCube, TouchCubeSparse) or 700 (CubeToBin)
steps; ``gym.make`` wraps the env in gymnasium's ``TimeLimit``, which sets ``truncated`` once the episode
reaches the limit (SO100Env.step itself always returns ``truncated=False``, env.py:180).  When gymnasium is
importable the ids are registered with it (``gym_so100/__init__.py``) and ``gym.make`` works as in the
reference; this module gives the same construction where it is absent (as in this image).
"""
from . import ENV_IDS
from .env import SO100Env


class TimeLimit:
    """gymnasium.wrappers.TimeLimit's contract: ``truncated = True`` on the step that reaches
    ``max_episode_steps`` since the last reset; everything else is the wrapped env's."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max_episode_steps = int(max_episode_steps)
        self._elapsed_steps = None

    def __getattr__(self, name):          # action_space, observation_space, render_mode, task, ...
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env

    def reset(self, seed=None, options=None):
        self._elapsed_steps = 0
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        if self._elapsed_steps is None:
            raise RuntimeError("Cannot call env.step() before calling env.reset()")
        obs, reward, terminated, truncated, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            truncated = True
        return obs, reward, terminated, truncated, info

    def render(self):
        return self.env.render()

    def close(self):
        return self.env.close()


def make(env_id, max_episode_steps=None, **kwargs):
    """``gym.make(env_id, **kwargs)`` for the reference's ids: SO100Env(task=..., obs_type=
    "so100_pixels_agent_pos", **kwargs) under a TimeLimit of the registered length."""
    if env_id not in ENV_IDS:
        raise ValueError(f"unknown env id {env_id!r}; registered: {sorted(ENV_IDS)}")
    spec = ENV_IDS[env_id]
    kw = dict(obs_type="so100_pixels_agent_pos", task=spec["task"])
    kw.update(kwargs)
    limit = spec["max_episode_steps"] if max_episode_steps is None else max_episode_steps
    return TimeLimit(SO100Env(**kw), limit)
