"""MI355X-native SO-ARM100 bin-a-cube simulator with the reference's gym_so100 API.

* ``SO100VecEnv``: batched envs on one GPU (torch tensors), the hot path.
* ``SO100Env`` / ``SO100GoalEnv``: single-env Gymnasium-style classes (reference env.py).
* Registration of the reference's env ids when gymnasium is importable (reference __init__.py:4-32), and
  ``gym_so100.make(id, **kwargs)``, the same construction (SO100Env + TimeLimit) where it is not.
"""
from .vec_env import SO100VecEnv  # noqa: F401
from .env import SO100Env, SO100GoalEnv  # noqa: F401

ENV_IDS = {
    "gym_so100/SO100TouchCube-v0": dict(max_episode_steps=300, task="so100_touch_cube"),
    "gym_so100/SO100TouchCubeSparse-v0": dict(max_episode_steps=300, task="so100_touch_cube_sparse"),
    "gym_so100/SO100CubeToBin-v0": dict(max_episode_steps=700, task="so100_cube_to_bin"),
}

try:  # gymnasium is an optional dependency here (absent in this image)
    from gymnasium.envs.registration import register as _register

    for _id, _kw in ENV_IDS.items():
        _register(id=_id, entry_point="gym_so100.env:SO100Env", max_episode_steps=_kw["max_episode_steps"],
                  nondeterministic=True, kwargs={"obs_type": "so100_pixels_agent_pos", "task": _kw["task"]})
except ImportError:
    pass

from .registration import make  # noqa: E402,F401  (gym.make for the ids above where gymnasium is absent)
