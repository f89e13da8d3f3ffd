"""The reference's own known-answer tests for the normalizers
(normalization.rs:373-690) and the empty-mask panic (utils.rs:246-254), ported
against the oracle — they pin the restatement the device's ObsNormalizer /
ReturnNormalizer paths are checked against (tests/test_gpu_*.py)."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O


class Obs:
    def __init__(self, dim, clip):
        self.n = O.ObsNorm()
        O.lib().or_obs_norm_init(C.byref(self.n), dim, clip)
        self.dim = dim

    def update(self, x):
        x = np.asarray(x, np.float32)
        O.lib().or_obs_norm_update_batch(C.byref(self.n), x, x.size // self.dim)

    def normalize(self, x):
        x = np.array(x, np.float32)
        O.lib().or_obs_norm_normalize_batch(C.byref(self.n), x, x.size // self.dim)
        return x

    mean = property(lambda s: [s.n.mean[j] for j in range(s.dim)])
    var = property(lambda s: [s.n.var[j] for j in range(s.dim)])
    count = property(lambda s: s.n.count)

    def __del__(self):
        O.lib().or_obs_norm_free(C.byref(self.n))


class Ret:
    def __init__(self, envs, players, gamma, clip):
        self.n = O.RetNorm()
        O.lib().or_ret_norm_init(C.byref(self.n), envs, players, gamma, clip)
        self.P = players

    def ret(self, e, p):
        return self.n.returns[e * self.P + p]

    def update_return(self, e, p, r):
        O.lib().or_ret_norm_update_return(C.byref(self.n), e, p, r)

    def update_variance_stats(self, e, p):
        O.lib().or_ret_norm_update_variance(C.byref(self.n), e, p)

    def reset_player(self, e, p):
        O.lib().or_ret_norm_reset_player(C.byref(self.n), e, p)

    def reset_env(self, e):
        O.lib().or_ret_norm_reset_env(C.byref(self.n), e)

    def normalize(self, r):
        return O.lib().or_ret_norm_normalize(C.byref(self.n), r)

    def variance(self):                              # normalization.rs:246-253
        return 0.0 if self.n.count < 2.0 else self.n.var / self.n.count

    def update_and_normalize_all(self, rewards, dones):
        r = np.array(rewards, np.float32)
        O.lib().or_ret_norm_update_and_normalize_all(C.byref(self.n), r, np.array(dones, np.uint8))
        return r

    def __del__(self):
        O.lib().or_ret_norm_free(C.byref(self.n))


# ------------------------------------------------------------ ObsNormalizer ---
def test_normalizer_update_and_normalize():          # normalization.rs:379-399
    n = Obs(2, 10.0)
    n.update([1.0, 2.0, 3.0, 4.0, 5.0, 6.0])
    assert abs(n.mean[0] - 3.0) < 0.1 and abs(n.mean[1] - 4.0) < 0.1
    t = n.normalize([3.0, 4.0])
    assert abs(t[0]) < 0.5 and abs(t[1]) < 0.5


def test_normalizer_clipping():                      # normalization.rs:401-415
    n = Obs(1, 5.0)
    n.update([0.0, 1.0, 0.0, 1.0])
    e = n.normalize([1000.0])
    assert -5.0 <= e[0] <= 5.0


def test_normalize_does_not_modify_stats():          # normalization.rs:417-436
    n = Obs(2, 10.0)
    n.update([1.0, 2.0, 3.0, 4.0, 5.0, 6.0])
    before = (n.count, n.mean, n.var)
    n.normalize([100.0, 200.0])
    assert (n.count, n.mean, n.var) == before


def test_normalize_with_insufficient_samples():      # normalization.rs:438-452
    n = Obs(2, 10.0)
    n.update([5.0, 10.0])
    assert n.count == 1.0
    assert list(n.normalize([3.0, 7.0])) == [3.0, 7.0]


def test_welford_correctness():                      # normalization.rs:454-468
    n = Obs(1, 10.0)
    n.update([1.0, 2.0, 3.0, 4.0, 5.0])
    assert abs(n.mean[0] - 3.0) < 1e-6
    assert abs(n.var[0] / n.count - 2.0) < 1e-6


def test_batch_update_equals_sequential():           # normalization.rs:470-490
    a, b = Obs(1, 10.0), Obs(1, 10.0)
    obs = [1.0, 2.0, 3.0, 4.0, 5.0]
    a.update(obs)
    for o in obs:
        b.update([o])
    assert abs(a.mean[0] - b.mean[0]) < 1e-10 and abs(a.var[0] - b.var[0]) < 1e-10 and a.count == b.count


def test_lagged_normalization_behavior():            # normalization.rs:492-524
    n = Obs(1, 10.0)
    n.update([0.0, 10.0])
    mean_before, var_before = n.mean[0], n.var[0]
    got = n.normalize([15.0])
    expected = (15.0 - mean_before) / np.sqrt(var_before / 2.0)
    assert abs(float(got[0]) - expected) < 0.01 and abs(expected - 2.0) < 1e-12
    n.update([15.0])
    assert n.count > 2.0 and abs(n.mean[0] - mean_before) > 0.1


# --------------------------------------------------------- ReturnNormalizer ---
def test_return_normalizer_rolling_return():         # normalization.rs:535-548
    n = Ret(2, 1, 0.99, 10.0)
    n.update_return(0, 0, 1.0)
    assert abs(n.ret(0, 0) - 1.0) < 1e-6
    n.update_return(0, 0, 1.0)
    assert abs(n.ret(0, 0) - 1.99) < 1e-6


def test_return_normalizer_reset_player():           # normalization.rs:550-561
    n = Ret(2, 1, 0.99, 10.0)
    n.update_return(0, 0, 10.0)
    assert n.ret(0, 0) > 0.0
    n.reset_player(0, 0)
    assert n.ret(0, 0) == 0.0


def _five_episodes(n):
    for r in [1.0, 2.0, 3.0, 4.0, 5.0]:
        n.update_return(0, 0, r)
        n.update_variance_stats(0, 0)
        n.reset_player(0, 0)


def test_return_normalizer_variance_stats():         # normalization.rs:563-579
    n = Ret(1, 1, 0.99, 10.0)
    _five_episodes(n)
    assert n.n.count == 5.0
    assert abs(n.variance() - 2.0) < 0.1


def test_return_normalizer_normalize():              # normalization.rs:581-598
    n = Ret(1, 1, 0.99, 10.0)
    _five_episodes(n)
    z = n.normalize(2.0)
    assert 0.0 < z < 10.0
    assert abs(z - 2.0 / np.sqrt(2.0 + 1e-8)) < 1e-6


def test_return_normalizer_clipping():               # normalization.rs:600-615
    n = Ret(1, 1, 0.99, 5.0)
    for _ in range(10):
        n.update_return(0, 0, 1.0)
        n.update_variance_stats(0, 0)
        n.reset_player(0, 0)
    z = n.normalize(100.0)
    assert -5.0 <= z <= 5.0


def test_return_normalizer_no_normalize_insufficient_samples():   # normalization.rs:617-628
    n = Ret(1, 1, 0.99, 10.0)
    n.update_return(0, 0, 5.0)
    n.update_variance_stats(0, 0)
    n.reset_player(0, 0)
    assert n.normalize(10.0) == 10.0


def test_return_normalizer_per_player_tracking():    # normalization.rs:630-648
    n = Ret(1, 2, 0.99, 10.0)
    n.update_return(0, 0, 1.0)
    assert abs(n.ret(0, 0) - 1.0) < 1e-6 and n.ret(0, 1) == 0.0
    n.update_return(0, 1, 2.0)
    assert abs(n.ret(0, 0) - 1.0) < 1e-6 and abs(n.ret(0, 1) - 2.0) < 1e-6
    n.update_return(0, 0, 1.0)
    assert abs(n.ret(0, 0) - 1.99) < 1e-6


def test_return_normalizer_reset_env():              # normalization.rs:650-665
    n = Ret(2, 2, 0.99, 10.0)
    n.update_return(0, 0, 1.0)
    n.update_return(0, 1, 2.0)
    n.update_return(1, 0, 3.0)
    n.reset_env(0)
    assert n.ret(0, 0) == 0.0 and n.ret(0, 1) == 0.0 and abs(n.ret(1, 0) - 3.0) < 1e-6


def test_return_normalizer_update_and_normalize_all():   # normalization.rs:667-690
    n = Ret(3, 1, 0.99, 10.0)
    n.update_and_normalize_all([1.0, 2.0, 3.0], [True, True, True])
    n.update_and_normalize_all([1.0, 2.0, 3.0], [True, True, True])
    r3 = n.update_and_normalize_all([2.0, 2.0, 2.0], [False, False, False])
    assert r3[0] > 0.0


# ------------------------------------------------------------ action masks ---
def test_apply_action_mask_neg_inf():                # utils.rs:231-244
    lg = np.zeros(4, np.float32)
    assert O.lib().or_apply_action_mask(lg, np.array([1, 0, 1, 0], np.uint8), 1, 4) == -1
    assert lg[0] == 0.0 and lg[2] == 0.0 and np.isneginf(lg[1]) and np.isneginf(lg[3])


def test_apply_action_mask_empty_row_panics():       # utils.rs:246-254 (#[should_panic])
    lg = np.zeros(6, np.float32)
    m = np.array([1, 1, 0, 0, 0, 0], np.uint8)      # row 1 of 2 (A = 3) has no valid action
    assert O.lib().or_apply_action_mask(lg, m, 2, 3) == 1
    assert (lg == 0.0).all()                         # nothing applied: the reference panics first


# --------------------------------------------------------------- PopArt ---
class Pop:
    def __init__(self):
        self.p = O.PopArt()
        O.lib().or_popart_init(C.byref(self.p))

    def update(self, xs):
        om, os_ = C.c_double(), C.c_double()
        O.lib().or_popart_update(C.byref(self.p), np.asarray(xs, np.float32), len(xs), C.byref(om), C.byref(os_))
        return om.value, os_.value

    def std(self):
        return O.lib().or_popart_std(C.byref(self.p))

    def initialized(self):
        return self.p.count >= 2.0

    def normalize(self, xs):
        x = np.asarray(xs, np.float32)
        out = np.zeros_like(x)
        O.lib().or_popart_normalize(C.byref(self.p), x, x.size, out)
        return out

    def denormalize(self, xs):
        x = np.array(xs, np.float32)
        O.lib().or_popart_denormalize(C.byref(self.p), x, x.size)
        return x


def test_popart_creation():                          # normalization.rs:713-718
    n = Pop()
    assert not n.initialized() and n.std() == 1.0


def test_popart_update():                            # normalization.rs:721-736
    n = Pop()
    _, os_ = n.update([10.0])
    assert not n.initialized() and os_ == 1.0
    n.update([20.0])
    assert n.initialized() and abs(n.p.mean - 15.0) < 0.01


def test_popart_multi_sample_update():               # normalization.rs:739-749
    n = Pop()
    n.update([0.0, 10.0, 20.0, 30.0, 40.0])
    assert abs(n.p.mean - 20.0) < 0.01 and 14.0 < n.std() < 15.0
    assert n.std() == np.sqrt(200.0 + 1e-4)


def test_popart_normalize():                         # normalization.rs:752-765
    n = Pop()
    n.update([0.0, 10.0, 20.0, 30.0, 40.0])
    assert abs(n.normalize([20.0])[0]) < 0.1
    assert 0.5 < n.normalize([34.14])[0] < 1.5


def test_popart_returns_old_stats():                 # normalization.rs:768-785
    n = Pop()
    n.update([0.0, 10.0])
    mb, sb = n.p.mean, n.std()
    om, os_ = n.update([20.0])
    assert abs(om - mb) < 1e-10 and abs(os_ - sb) < 1e-10 and n.p.mean != mb


def test_popart_normalize_before_initialized():      # normalization.rs:800-810
    n = Pop()
    n.update([10.0])
    assert not n.initialized() and n.normalize([5.0])[0] == 5.0


def test_popart_denormalize_inverse_of_normalize():  # normalization.rs:813-827
    n = Pop()
    n.update([10.0, 20.0, 100.0, 200.0])
    d = n.denormalize(n.normalize([15.0, 150.0]))
    assert np.allclose(d, [15.0, 150.0], atol=1e-4)


def test_popart_denormalize_before_initialized():    # normalization.rs:830-841
    n = Pop()
    n.update([10.0])
    assert n.denormalize([5.0])[0] == 5.0
