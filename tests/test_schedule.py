"""Schedule::get (schedule.rs:54-78) — the reference's own known answers
(schedule.rs:283-523) against the oracle restatement (oracle/vecenv.c
or_schedule_get), the host mirror (bppo.host.schedule_get, used for the learning
rate / entropy schedules) and the device's restatement through its config forms.
The device-side evaluation (bppo_internal.h schedule_get, Liar's Dice shaping) is
checked on the GPU in tests/test_gpu_wide.py::test_liars_dice_shaping_schedule."""
import numpy as np
import pytest

import oracle_ffi as O
from bppo.host import make_config, schedule_get, shaping_schedule, to_struct


def _oracle(ms, step):
    v = np.ascontiguousarray([a for a, _ in ms], np.float64)
    s = np.ascontiguousarray([b for _, b in ms], np.uint64)
    return O.lib().or_schedule_get(v.ctypes.data, s.ctypes.data, len(ms), step)


def _both(ms, step):
    a, b = _oracle(ms, step), schedule_get(ms, step)
    assert a == b
    return a


KNOWN = [  # (milestones, step, expected) — schedule.rs test_* cases (exact asserts)
    ([(0.001, 0)], 0, 0.001), ([(0.001, 0)], 1_000_000, 0.001), ([(0.001, 0)], 100_000_000, 0.001),
    ([(1.0, 0), (0.0, 100)], 0, 1.0), ([(1.0, 0), (0.0, 100)], 50, 0.5), ([(1.0, 0), (0.0, 100)], 100, 0.0),
    ([(1.0, 0), (0.0, 100)], 200, 0.0),
    ([(1.0, 0), (0.5, 100), (0.1, 200)], 0, 1.0), ([(1.0, 0), (0.5, 100), (0.1, 200)], 50, 0.75),
    ([(1.0, 0), (0.5, 100), (0.1, 200)], 100, 0.5), ([(1.0, 0), (0.5, 100), (0.1, 200)], 150, 0.3),
    ([(1.0, 0), (0.5, 100), (0.1, 200)], 200, 0.1), ([(1.0, 0), (0.5, 100), (0.1, 200)], 300, 0.1),
    ([(0.0, 0), (1.0, 100)], 0, 0.0), ([(0.0, 0), (1.0, 100)], 50, 0.5), ([(0.0, 0), (1.0, 100)], 100, 1.0),
    ([(1.0, 0), (1.0, 100), (0.0, 200)], 50, 1.0), ([(1.0, 0), (1.0, 100), (0.0, 200)], 150, 0.5),
    ([(0.5, 1000)], 0, 0.5), ([(0.5, 1000)], 999, 0.5), ([(0.5, 1000)], 1000, 0.5), ([(0.5, 1000)], 2000, 0.5),
    ([], 0, 0.0), ([], 1000, 0.0),
    ([(1.0, 0), (0.0, 1_000_000_000)], 500_000_000, 0.5), ([(1.0, 0), (0.0, 1_000_000_000)], 1_000_000_000, 0.0),
    ([(1.0, 0), (0.0, 1_000_000_000)], 2_000_000_000, 0.0),
    ([(0.001, 0), (0.0001, 100)], 0, 0.001), ([(0.5, 100)], 0, 0.5),
]


@pytest.mark.parametrize("ms,step,want", KNOWN)
def test_schedule_known_answers(ms, step, want):
    assert _both(ms, step) == want


def test_schedule_boundary_conditions():
    s = [(1.0, 0), (0.0, 100)]                      # schedule.rs:505-515
    assert abs(_both(s, 1) - 0.99) < 0.001
    assert abs(_both(s, 99) - 0.01) < 0.001


def test_schedule_halfway_doc_example():
    assert _both([(0.001, 0), (0.0001, 30_000_000)], 15_000_000) == 0.00055   # schedule.rs:16-18


def test_shaping_config_forms():
    # a number is Schedule::constant; a list is sorted by step (schedule.rs:232-270, 474-485)
    assert shaping_schedule(make_config("liars_dice_ctde")) == [(0.05, 0)]
    c = make_config("liars_dice_ctde", reward_shaping_coef=[(0.0001, 30_000_000), (0.001, 0)])
    assert shaping_schedule(c) == [(0.001, 0), (0.0001, 30_000_000)]
    assert to_struct(c).reward_shaping_coef == 0.001      # initial value in the config struct
