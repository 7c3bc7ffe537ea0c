"""Task constants and action scaling for the SO-ARM100 envs (host-side mirror of the reference API).

Mirrors the public names of /root/reference/gym_so100/constants.py so reference users find them;
the batched hot path applies the same scaling inside the HIP step kernel prologue
(csrc/so100_step.hip, ``unnormalize_f32``).
"""
from pathlib import Path

import numpy as np

DT = 0.02            # control period (constants.py:4)  -> 10 physics substeps of 0.002 s
FPS = 50             # constants.py:5

SO100_JOINTS = ["left_arm_waist", "left_arm_shoulder", "left_arm_elbow", "left_arm_forearm_roll",
                "left_arm_wrist_rotate", "left_arm_gripper"]           # constants.py:8-16
SO100_ACTIONS = list(SO100_JOINTS)                                   # constants.py:18-26

# GoalEnv bin box (constants.py:29-30)
bin_min = np.array([-0.25, 0.7, 0.01], dtype=np.float32)
bin_max = np.array([-0.14, 0.76, 0.05], dtype=np.float32)

SO100_START_ARM_POSE = [0.0, -0.96, 1.16, 0.0, 0.0, 0.02239]          # constants.py:32-39

# per-joint (low, high) of unnormalize_so100 (constants.py:78-86) == the MJCF joint ranges
SO100_ACTION_RANGES = [(-1.92, 1.92), (-3.32, 0.174), (-0.174, 3.14), (-1.66, 1.66), (-2.79, 2.79),
                       (-0.174, 1.75)]

# sample_so100_box_pose ranges (utils.py:18-22)
SO100_BOX_SPAWN_RANGES = [(-0.25, -0.15), (0.3, 0.6), (0.05, 0.05)]

# SO100Task._precompute_bin_aabb (single_arm.py:69-75)
BIN_HALF_WIDTH = 0.06
BIN_INNER_HEIGHT = 0.03
CUBE_HALF = 0.01
MAX_REWARD = 4.0                      # single_arm.py:130,227,297
GOAL_DISTANCE_THRESHOLD = 0.01        # env.py:252
GOAL_CURRICULUM_STEPS = 5000          # env.py:324
GOAL_MAX_EPISODE_STEPS = 300          # env.py:200

ASSETS_DIR = Path(__file__).parent.resolve() / "assets"


def unnormalize(num, min_val, max_val, original_min=-1, original_max=1):
    """Affine map [original_min, original_max] -> [min_val, max_val], then clip (constants.py:44-47)."""
    span = original_max - original_min
    out = (num - original_min) / span * (max_val - min_val) + min_val
    return np.clip(out, min_val, max_val)


def normalize(num, min_val, max_val, target_min=-1, target_max=1):
    """Inverse map [min_val, max_val] -> [target_min, target_max], clipped (constants.py:71-76)."""
    if min_val == max_val:
        return 0.0
    out = (num - min_val) / (max_val - min_val) * (target_max - target_min) + target_min
    return np.clip(out, target_min, target_max)


def unnormalize_so100(action):
    """In-place per-joint un-normalisation of a 6-vector (constants.py:78-86)."""
    for k, (lo, hi) in enumerate(SO100_ACTION_RANGES):
        action[k] = unnormalize(action[k], lo, hi)
    return action


def normalize_so100(action):
    """In-place per-joint normalisation to [-1, 1] (constants.py:49-57)."""
    for k, (lo, hi) in enumerate(SO100_ACTION_RANGES):
        action[k] = normalize(action[k], lo, hi)
    return action


_LEROBOT_RANGES = [(-100, 100)] * 5 + [(0, 100)]                      # constants.py:60-68,89-96


def normalize_gym_so100_to_lerobot(action):
    for k, ((lo, hi), (tlo, thi)) in enumerate(zip(SO100_ACTION_RANGES, _LEROBOT_RANGES)):
        action[k] = normalize(action[k], lo, hi, tlo, thi)
    return action


def normalize_lerobot_to_gym_so100(action):
    for k, (lo, hi) in enumerate(_LEROBOT_RANGES):
        action[k] = normalize(action[k], lo, hi)
    return action
