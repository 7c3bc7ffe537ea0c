"""Demonstration formats of the reference, recorded from batched GPU envs.

* ``DemoRecorder`` writes episodes in the layout of the reference's expert demonstrations
  (scripts/record_teleop.py:163-184, 257-284, saved with pickle by ``save_demonstrations``): a list of
  episodes, each ``{"observations", "actions", "rewards", "infos"}`` lists with one entry per step, as an
  SB3 VecEnv of one env (``VecTransposeImage`` + ``VecNormalize(norm_obs=False)``, record_teleop.py:137-153)
  hands them over: observation ``{"pixels": uint8 [1, 3, H, W], "agent_pos": float32 [1, 6]}`` (the
  observation returned by the step), action float32 [6], reward float32 [1], info ``[dict]``.
  N envs are recorded at once; an episode ends at terminated or truncated.
* ``lerobot_frames`` turns an episode into the frame dicts that scripts/upload_lerobot_demos.py:192-201
  passes to ``LeRobotDataset.add_frame`` (LeRobot itself is not installed here).
* ``load_demonstrations`` reads such a file with an unpickler restricted to numpy arrays and builtins.
"""
import io
import pickle

import numpy as np

FPS = 50                                    # gym_so100/constants.py:5


def _torch():
    import torch
    return torch


class DemoRecorder:
    """Collect episodes from an ``SO100VecEnv`` with ``obs_type="so100_pixels_agent_pos"``.

    Call ``add(actions, obs, reward, terminated, truncated, info)`` after every ``venv.step(actions)``;
    finished episodes accumulate in ``demonstrations`` (the reference's list), ``env_ids`` limits the
    recorded envs."""

    def __init__(self, venv, env_ids=None, max_episodes=None):
        if venv.renderer is None:
            raise ValueError("DemoRecorder needs obs_type='so100_pixels_agent_pos' (record_teleop.py:127-133)")
        self.venv = venv
        self.env_ids = list(range(venv.num_envs)) if env_ids is None else [int(i) for i in env_ids]
        self.max_episodes = max_episodes
        self.demonstrations = []
        self._cur = {i: self._empty() for i in self.env_ids}

    @staticmethod
    def _empty():
        return {"observations": [], "actions": [], "rewards": [], "infos": []}

    @property
    def done(self):
        return self.max_episodes is not None and len(self.demonstrations) >= self.max_episodes

    def add(self, actions, obs, reward, terminated, truncated, info):
        torch = _torch()
        ids = torch.as_tensor(self.env_ids, device=self.venv.device)
        # one device->host copy per field for the recorded envs; pixels to channel-first like
        # VecTransposeImage
        pix = obs["pixels"].index_select(0, ids).permute(0, 3, 1, 2).contiguous().cpu().numpy()
        pos = obs["agent_pos"].index_select(0, ids).cpu().numpy().astype(np.float32)
        act = torch.as_tensor(actions).to(self.venv.device, torch.float32).index_select(0, ids).cpu().numpy()
        rew = reward.index_select(0, ids).cpu().numpy().astype(np.float32)
        term = terminated.index_select(0, ids).cpu().numpy()
        trunc = truncated.index_select(0, ids).cpu().numpy()
        succ = info["is_success"].index_select(0, ids).cpu().numpy()
        for k, i in enumerate(self.env_ids):
            ep = self._cur[i]
            ep["observations"].append({"pixels": pix[k:k + 1].copy(), "agent_pos": pos[k:k + 1].copy()})
            ep["actions"].append(act[k].copy())
            ep["rewards"].append(rew[k:k + 1].copy())
            step_info = {"is_success": bool(succ[k])}
            if trunc[k] and not term[k]:
                step_info["TimeLimit.truncated"] = True
            ep["infos"].append([step_info])
            if term[k] or trunc[k]:
                if not self.done:
                    self.demonstrations.append(ep)
                self._cur[i] = self._empty()

    def save(self, filename="expert_demonstrations.pkl"):
        """record_teleop.py:277-284: pickle.dump of the episode list."""
        with open(filename, "wb") as f:
            pickle.dump(self.demonstrations, f)
        return filename


class _NumpyUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
                ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar"), ("builtins", "dict"), ("builtins", "list")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"demonstration files may only hold numpy arrays: {module}.{name}")


def load_demonstrations(filename):
    """Read a demonstrations file (upload_lerobot_demos.py:36-45) without executing code from it."""
    with open(filename, "rb") as f:
        return _NumpyUnpickler(io.BytesIO(f.read())).load()


def lerobot_frames(episode):
    """The frame dicts upload_lerobot_demos.py:120-201 builds from one episode (same keys, shapes, dtypes)."""
    obs, acts, rews = episode["observations"], episode["actions"], episode["rewards"]
    n = min(len(obs), len(acts))
    frames = []
    for i in range(n):
        pixels = np.asarray(obs[i]["pixels"])
        image = pixels[0] if pixels.ndim == 4 and pixels.shape[0] == 1 else pixels
        pos = np.asarray(obs[i]["agent_pos"], np.float32)
        state = pos[0] if pos.ndim == 2 and pos.shape[0] == 1 else pos
        reward = np.asarray(rews[i] if i < len(rews) else [0.0], np.float32)
        frames.append({"observation.state": state.astype(np.float32),
                       "observation.images.top": image,
                       "action": np.asarray(acts[i], np.float32).reshape(-1),
                       "next.reward": np.array([reward.reshape(-1)[0]], np.float32)[0],
                       "next.success": np.array([reward.squeeze() >= 4], np.bool_),
                       "seed": np.array([0], np.int64),
                       "timestamp": np.float32(i / FPS)})
    return frames
