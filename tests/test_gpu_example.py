"""configs[0] (BASELINE.json): the reference's scripts/example.py:10-28 loop on this build, driven through
tools/example.py -- TouchCube, so100_pixels_agent_pos at 64x48, 1000 random-action steps across episode
boundaries (the registered TimeLimit of 300), render() every step -- with the properties that loop implies."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


def test_example_loop_1000_steps():
    import example
    from gym_so100.constants import SO100_JOINTS  # noqa: F401
    from gym_so100.model import build_model
    frames, log = example.run(1000, seed=7)
    assert frames.shape == (1000, 48, 64, 3) and frames.dtype == np.uint8
    assert all(r["image_shape"] == (480, 640, 3) for r in log)          # render(): visualization size
    m = build_model()
    lo = np.array([m.jnt_range[j][0] for j in range(6)]) - 0.05
    hi = np.array([m.jnt_range[j][1] for j in range(6)]) + 0.05
    ep_len, lengths, ends = 0, [], []
    for t, r in enumerate(log):
        q = r["agent_pos"]
        assert q.shape == (6,) and q.dtype == np.float32 and np.all(np.isfinite(q))
        assert np.all(q >= lo) and np.all(q <= hi), (t, q)               # joint limits (soft, +- 0.05 rad)
        rew = r["reward"]
        assert isinstance(rew, float) and -0.2 - 1e-12 <= rew <= 4.0       # TouchCube ladder range
        assert r["terminated"] == (rew == 4.0) == r["info"]["is_success"]  # env.py:176
        c = r["cube"]
        assert np.all(np.isfinite(c)) and c[2] > -0.01 and abs(np.linalg.norm(c[3:]) - 1) < 1e-5
        ep_len += 1
        if r["terminated"] or r["truncated"]:
            lengths.append(ep_len)
            ends.append("term" if r["terminated"] else "trunc")
            ep_len = 0
    assert len(lengths) >= 3, lengths                                     # 1000 steps cross episode ends
    for n, kind in zip(lengths, ends):
        assert n <= 300 and (kind == "term" or n == 300), (lengths, ends)  # TimeLimit 300 (__init__.py:7)
    # each episode starts from the start pose (single_arm.py:132-142): the first step moves < 0.2 rad
    from gym_so100.constants import SO100_START_ARM_POSE as START_ARM_POSE
    starts = [0] + [i + 1 for i, r in enumerate(log[:-1]) if r["terminated"] or r["truncated"]]
    for s in starts:
        assert np.max(np.abs(log[s]["agent_pos"] - np.asarray(START_ARM_POSE[:6], np.float32))) < 0.2
    # the frames change with the state and are not blank
    assert frames.reshape(1000, -1).std(axis=1).min() > 1.0
    assert np.abs(frames[1:].astype(int) - frames[:-1].astype(int)).sum() > 0


def test_example_loop_is_deterministic_with_a_seed():
    import example
    f1, l1 = example.run(120, seed=3)
    f2, l2 = example.run(120, seed=3)
    np.testing.assert_array_equal(f1, f2)
    assert [r["reward"] for r in l1] == [r["reward"] for r in l2]
