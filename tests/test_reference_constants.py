"""The reference's own known-answer tests (tests/test_constants.py:6-35), restated against our mirror."""
import numpy as np

from gym_so100.constants import normalize, unnormalize, SO100_ACTION_RANGES, SO100_START_ARM_POSE, DT


def test_unnormalize_known_answers():
    cases = [(-1, -10, 10, -10), (1, -10, 10, 10), (0, -10, 10, 0), (0.5, -10, 10, 5), (-0.5, -10, 10, -5),
             (-2, -10, 10, -10), (2, -10, 10, 10), (0, 0, 20, 10), (-1, 0, 20, 0), (1, 0, 20, 20)]
    for num, lo, hi, want in cases:
        assert unnormalize(num, lo, hi) == want
    assert np.isclose(unnormalize(0.25, -5.0, 5.0), 1.25)


def test_normalize_inverts_unnormalize():
    for lo, hi in SO100_ACTION_RANGES:
        for a in np.linspace(-1, 1, 9):
            assert np.isclose(normalize(unnormalize(a, lo, hi), lo, hi), a)
    assert normalize(3.0, 1.0, 1.0) == 0.0


def test_task_constants():
    assert DT == 0.02
    assert SO100_START_ARM_POSE == [0.0, -0.96, 1.16, 0.0, 0.0, 0.02239]
