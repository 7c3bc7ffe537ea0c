"""Demonstration file format (scripts/record_teleop.py, scripts/upload_lerobot_demos.py)."""
import os
import pickle

import numpy as np
import pytest

from gym_so100.demos import lerobot_frames, load_demonstrations


def synthetic_episode(T=5, H=6, W=8):
    rng = np.random.default_rng(0)
    ep = {"observations": [], "actions": [], "rewards": [], "infos": []}
    for t in range(T):
        ep["observations"].append({"pixels": rng.integers(0, 255, (1, 3, H, W), dtype=np.uint8),
                                   "agent_pos": rng.normal(size=(1, 6)).astype(np.float32)})
        ep["actions"].append(rng.uniform(-1, 1, 6).astype(np.float32))
        ep["rewards"].append(np.array([4.0 if t == T - 1 else 1.0], np.float32))
        ep["infos"].append([{"is_success": t == T - 1}])
    return ep


def test_round_trip_and_frames(tmp_path):
    eps = [synthetic_episode(), synthetic_episode(3)]
    p = os.path.join(tmp_path, "demos.pkl")
    with open(p, "wb") as f:
        pickle.dump(eps, f)
    back = load_demonstrations(p)
    assert len(back) == 2 and len(back[0]["observations"]) == 5
    np.testing.assert_array_equal(back[0]["observations"][2]["pixels"], eps[0]["observations"][2]["pixels"])
    fr = lerobot_frames(back[0])
    assert len(fr) == 5
    f0 = fr[0]
    assert f0["observation.images.top"].shape == (3, 6, 8) and f0["observation.images.top"].dtype == np.uint8
    assert f0["observation.state"].shape == (6,) and f0["observation.state"].dtype == np.float32
    assert f0["action"].shape == (6,) and f0["action"].dtype == np.float32
    assert f0["next.reward"] == np.float32(1.0) and not f0["next.success"][0]
    assert fr[-1]["next.success"][0] and fr[-1]["next.reward"] == 4.0
    assert f0["seed"].dtype == np.int64 and fr[1]["timestamp"] == np.float32(1 / 50)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_loader_executes_nothing(tmp_path):
    p = os.path.join(tmp_path, "evil.pkl")
    with open(p, "wb") as f:
        pickle.dump([{"observations": [_Evil()]}], f)
    with pytest.raises(pickle.UnpicklingError):
        load_demonstrations(p)
