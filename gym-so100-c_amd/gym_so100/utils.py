"""Host-side spawn helpers with the reference's names (gym_so100/utils.py).

The batched env computes spawns on the device (csrc/so100_step.hip ``spawn_pose``: numpy legacy
MT19937 restated); these numpy versions are kept for API compatibility and for host-side users.
"""
import numpy as np

from .constants import SO100_BOX_SPAWN_RANGES


def _pose(ranges, seed):
    rng = np.random.RandomState(seed)
    r = np.asarray(ranges, dtype=np.float64)
    return np.concatenate([rng.uniform(r[:, 0], r[:, 1]), [1.0, 0.0, 0.0, 0.0]])


def sample_so100_box_pose(seed=None):
    """Cube pose: x in [-0.25,-0.15], y in [0.3,0.6], z = 0.05, identity quaternion (utils.py:18-29)."""
    return _pose(SO100_BOX_SPAWN_RANGES, seed)


def sample_box_pose(seed=None):
    """utils.py:4-15."""
    return _pose([(0.0, 0.2), (0.4, 0.6), (0.05, 0.05)], seed)


def fixed_so100_box_pose(seed=None):
    """utils.py:32-40."""
    return np.array([-0.2, 0.45, 0.05, 1.0, 0.0, 0.0, 0.0])
