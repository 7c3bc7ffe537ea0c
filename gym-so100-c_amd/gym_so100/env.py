"""Single-env classes with the reference's constructor/reset/step API (gym_so100/env.py).

``SO100Env`` (env.py:26-185) and ``SO100GoalEnv`` (env.py:188-409) are thin views over a one-env
``SO100VecEnv`` on the GPU: numpy in, numpy out, like the reference.  For throughput use
``SO100VecEnv`` directly (thousands of envs per launch).

Observations: ``obs_type="so100_pixels_agent_pos"`` (the registered envs' and GoalEnv's form: the
``top`` camera drawn by the GPU rasteriser, render.py) or ``"so100_state"``.  ``render()`` draws the
same camera at the visualization size.  The images are the scene's geometry and colours, not MuJoCo's
OpenGL pixels.
"""
import numpy as np

from . import spaces
from .constants import SO100_ACTIONS, SO100_JOINTS, GOAL_DISTANCE_THRESHOLD, bin_max, bin_min
from .vec_env import SO100VecEnv
from .render import CameraRenderer

try:
    import gymnasium as _gym
    _Base = _gym.Env
except ImportError:          # gymnasium is optional here
    class _Base:
        metadata = {}

        def reset(self, seed=None, options=None):
            return None


def _check_seed(seed):
    """numpy.random.RandomState(seed) accepts integers in [0, 2**32) (utils.py:24); so does the cube spawn."""
    s = int(seed)
    if not 0 <= s < 2 ** 32:
        raise ValueError(f"Seed must be between 0 and 2**32 - 1 (got {seed})")
    return s


class SO100Env(_Base):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 50}

    def __init__(self, task, obs_type="pixels", render_mode="rgb_array", observation_width=640,
                 observation_height=480, visualization_width=640, visualization_height=480, device="cuda:0",
                 max_episode_steps=0, solver="newton"):
        """Same signature and default as the reference (env.py:28-38).  Its default obs_type "pixels" is
        one the reference's own code does not handle: no observation_space is set (env.py:50-73) and
        _format_raw_obs leaves `obs` unbound (env.py:130-146), so its first reset fails.  Here that default
        fails at construction, with the two obs types the reference does serve named; the registered ids
        (gym_so100/__init__.py:4-32) pass so100_pixels_agent_pos, as in the reference."""
        super().__init__()
        if obs_type not in ("so100_state", "so100_pixels_agent_pos"):
            raise ValueError(f"obs_type={obs_type!r} is not served (the reference's default 'pixels' fails "
                             "in its own _format_raw_obs, env.py:130-146): pass obs_type="
                             "'so100_pixels_agent_pos' (the registered envs') or 'so100_state'")
        self.task = task
        self.obs_type = obs_type
        self.render_mode = render_mode
        self.observation_width, self.observation_height = observation_width, observation_height
        self.visualization_width, self.visualization_height = visualization_width, visualization_height
        # TimeLimit is applied by the gymnasium registry wrapper (as in the reference); 0 = none here
        self._venv = SO100VecEnv(1, task=task, obs_type=obs_type, device=device, autoreset=False,
                                 max_episode_steps=max_episode_steps, solver=solver,
                                 observation_width=observation_width, observation_height=observation_height,
                                 reward64=True)
        self._vis = None
        if obs_type == "so100_pixels_agent_pos":                          # env.py:50-66
            self.observation_space = spaces.Dict({
                "pixels": spaces.Box(low=0, high=255, shape=(observation_height, observation_width, 3),
                                     dtype=np.uint8),
                "agent_pos": spaces.Box(low=-10.0, high=10.0, shape=(len(SO100_JOINTS),), dtype=np.float32)})
        else:
            self.observation_space = spaces.Box(low=-100.0, high=100.0, shape=(len(SO100_JOINTS) + 3 * 3,),
                                                dtype=np.float32)       # env.py:67-73
        self.action_space = spaces.Box(low=-1, high=1, shape=(len(SO100_ACTIONS),), dtype=np.float32)

    def reset(self, seed=None, options=None):
        """seed: an int in [0, 2**32) spawns the cube as numpy's RandomState(seed) (utils.py:18-29, which rejects
        other values); None draws a fresh spawn (in-kernel seed from the env's base seed and episode counter,
        where the reference's RandomState(None) draws from OS entropy)."""
        super().reset(seed=seed)
        obs, _ = self._venv.reset(seed=None if seed is None else [_check_seed(seed)])
        return self._np_obs(obs), {"is_success": False}                 # env.py:169

    def _np_obs(self, obs):
        if isinstance(obs, dict):
            return {k: v[0].cpu().numpy() for k, v in obs.items()}
        return obs[0].cpu().numpy()

    def step(self, action):
        action = np.asarray(action, dtype=np.float32)
        assert action.ndim == 1                                          # env.py:173
        obs, reward, terminated, truncated, info = self._venv.step(action[None, :6])
        r = float(self._venv.reward64[0].item())                       # float64, as the reference
        is_success = bool(info["is_success"][0].item())
        return self._np_obs(obs), r, bool(terminated[0].item()), False, {"is_success": is_success}

    def render(self):
        """Top camera at the visualization size (env.py:79-90), uint8 [H, W, 3]."""
        assert self.render_mode == "rgb_array"
        if self._vis is None:
            self._vis = CameraRenderer(self._venv, self.visualization_width, self.visualization_height)
        return self._vis.render()[0].cpu().numpy()

    def close(self):
        self._venv.close()


class SO100GoalEnv(_Base):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 50}

    def __init__(self, render_mode="rgb_array", observation_width=640, observation_height=480,
                 visualization_width=640, visualization_height=480, device="cuda:0", solver="newton",
                 obs_type="so100_pixels_agent_pos"):
        """obs_type "so100_pixels_agent_pos" (the reference's only form): "observation" = flattened
        pixels / 255 + agent_pos (env.py:218-224, 267-270); "so100_state": the 15-float state vector."""
        super().__init__()
        self.max_episode_steps = 300                                     # env.py:200
        self.current_step = 0
        self.render_mode = render_mode
        self.observation_width, self.observation_height = observation_width, observation_height
        self.visualization_width, self.visualization_height = visualization_width, visualization_height
        self._venv = SO100VecEnv(1, task="so100_goal", device=device, autoreset=False, solver=solver,
                                 obs_type=obs_type, observation_width=observation_width,
                                 observation_height=observation_height, reward64=True)
        self._vis = None
        self.distance_threshold = GOAL_DISTANCE_THRESHOLD                # env.py:252
        size = observation_height * observation_width * 3 + len(SO100_JOINTS) \
            if obs_type == "so100_pixels_agent_pos" else 15
        obs_space = spaces.Box(low=-np.inf, high=np.inf, shape=(size,), dtype=np.float32)
        self.observation_space = spaces.Dict({
            "observation": obs_space,
            "achieved_goal": spaces.Box(low=-np.inf, high=np.inf, shape=(3,), dtype=np.float32),
            "desired_goal": spaces.Box(low=-np.inf, high=np.inf, shape=(3,), dtype=np.float32)})
        self.action_space = spaces.Box(low=-1, high=1, shape=(len(SO100_ACTIONS),), dtype=np.float32)
        self.bin_goal_space = spaces.Box(low=np.array([bin_min[0] + 0.005, bin_min[1] + 0.005, 0.01]),
                                         high=np.array([bin_max[0] - 0.005, bin_max[1] - 0.005, 0.05]),
                                         dtype=np.float32)               # env.py:245-249

    @property
    def total_steps(self):
        return int(self._venv.total_steps[0].item())

    def _goal_obs(self, o):
        return {k: v[0].cpu().numpy() for k, v in o.items()}

    def reset(self, seed=None, options=None):
        super().reset(seed=seed)
        self.current_step = 0
        obs, _ = self._venv.reset(seed=None if seed is None else [_check_seed(seed)])
        return self._goal_obs(obs), {"is_success": False}

    def compute_reward(self, achieved_goal, desired_goal, info):
        """Sparse reward (env.py:341-353): batched -> float32 array, single -> python float."""
        a = np.asarray(achieved_goal)
        d = np.asarray(desired_goal)
        if a.ndim > 1:
            return self._venv.compute_reward(a, d).cpu().numpy()
        return 0.0 if np.linalg.norm(a - d) < self.distance_threshold else -1.0

    def step(self, action):
        action = np.asarray(action, dtype=np.float32)
        assert action.ndim == 1                                          # env.py:375
        obs, reward, terminated, truncated, info = self._venv.step(action[None, :6])
        self.current_step += 1
        out = self._goal_obs(obs)
        success = bool(info["is_success"][0].item())
        trunc = bool(truncated[0].item())
        inf = {"is_success": success}
        if trunc:
            inf["TimeLimit.truncated"] = True
        return out, float(self._venv.reward64[0].item()), bool(terminated[0].item()), trunc, inf

    def render(self):
        """Top camera at the visualization size (env.py:256-265), uint8 [H, W, 3]."""
        assert self.render_mode == "rgb_array"
        if self._vis is None:
            self._vis = CameraRenderer(self._venv, self.visualization_width, self.visualization_height)
        return self._vis.render()[0].cpu().numpy()

    def close(self):
        self._venv.close()
