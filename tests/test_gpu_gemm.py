"""The f32 MFMA GEMM engine (k_gemm.hip) through bppo_debug_gemm.

Forward (Burn Linear, mlp.rs:140-206) must be BIT-EXACT against the oracle's
matrixmultiply restatement (or_linear: k-ordered fma chains restarted at every
KC=256 block, blocks summed, then + bias): v_mfma_f32_32x32x2_f32 is itself a
k-ordered fmaf chain.  The backward forms (dX = dZ W^T masked by relu', dW =
X^T dZ with bias column sums) are checked against float64 numpy at 1e-5
relative of the row-sum of |products| (their summation order is free)."""
import numpy as np
import pytest

import bppo._lib as L
import oracle_ffi as O

pytestmark = pytest.mark.gpu


def _gemm(mode, M, N, K, A, B, X, relu=0):
    out = np.zeros((M, N), np.float32)
    out2 = np.zeros(N, np.float32)
    st = L.lib().bppo_debug_gemm(mode, M, N, K, L.ptr(A), L.ptr(B), None if X is None else L.ptr(X), relu,
                                 L.ptr(out), L.ptr(out2))
    assert st == 0
    return out, out2


# the shapes of the wide nets: C4 86->512->512->{7+1}, LD actor 270->256->256->49,
# LD critic 390->512->512->512->1, plus ragged edges
FWD_SHAPES = [(257, 512, 86), (300, 512, 512), (129, 8, 512), (64, 256, 270), (200, 49, 256),
              (100, 512, 390), (33, 1, 512), (1, 5, 3), (130, 130, 600)]


@pytest.mark.parametrize("M,N,K", FWD_SHAPES)
@pytest.mark.parametrize("relu", [1, -1])
def test_gemm_forward_bit_exact(M, N, K, relu):
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    X = rng.standard_normal((M, K)).astype(np.float32)
    if K == 86:   # one-hot boards, like Connect Four observations
        X = (rng.random((M, K)) < 0.3).astype(np.float32)
    W = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    y_ref = O.linear(X, W, b, relu)
    y, _ = _gemm(0, M, N, K, X, W, b, relu=1 if relu == 1 else 0)
    assert np.array_equal(y, y_ref), f"max |diff| {np.abs(y - y_ref).max()}"


@pytest.mark.parametrize("M,N,K", [(257, 512, 86), (300, 512, 512), (33, 130, 600)])
def test_gemm_forward_tanh_bit_exact(M, N, K):
    """tanh hidden layers (config.rs:990-992 default): GEMM + elementwise glibc tanhf"""
    rng = np.random.default_rng(M + 5 * N + K)
    X = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((K, N)) / np.sqrt(K) * 2.0).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    y_ref = O.linear(X, W, b, 0)          # oracle act 0 = tanhf
    y, _ = _gemm(0, M, N, K, X, W, b, relu=2)
    assert np.array_equal(y.view(np.uint32), y_ref.view(np.uint32))


@pytest.mark.parametrize("M,N,K", [(300, 512, 512), (129, 86, 8)])
def test_gemm_dx_tanh(M, N, K):
    rng = np.random.default_rng(M + N + K + 1)
    dZ = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)
    H = np.tanh(rng.standard_normal((M, N))).astype(np.float32)
    g = (dZ.astype(np.float64) @ W.astype(np.float64).T)
    mag = np.abs(dZ.astype(np.float64)) @ np.abs(W.astype(np.float64)).T
    ref = g * (1.0 - H.astype(np.float64) ** 2)
    out, _ = _gemm(1, M, N, K, dZ, W, H, relu=2)
    assert np.all(np.abs(out - ref) <= 2e-5 * mag + 1e-30)


@pytest.mark.parametrize("M,N,K", [(300, 512, 512), (257, 86, 512), (100, 256, 49), (70, 512, 1),
                                   (129, 512, 8)])
def test_gemm_dx(M, N, K):
    rng = np.random.default_rng(M + N + K)
    dZ = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)
    H = rng.standard_normal((M, N)).astype(np.float32)
    ref = (dZ.astype(np.float64) @ W.astype(np.float64).T) * (H > 0)
    mag = np.abs(dZ.astype(np.float64)) @ np.abs(W.astype(np.float64)).T
    out, _ = _gemm(1, M, N, K, dZ, W, H)
    assert np.all(np.abs(out - ref) <= 1e-5 * mag + 1e-30)
    out, _ = _gemm(1, M, N, K, dZ, W, None)
    ref = dZ.astype(np.float64) @ W.astype(np.float64).T
    assert np.all(np.abs(out - ref) <= 1e-5 * mag + 1e-30)


@pytest.mark.parametrize("Kin,N,rows", [(512, 512, 5000), (86, 512, 4099), (256, 49, 3000), (512, 1, 2500),
                                        (390, 512, 70000), (64, 8, 31)])
def test_gemm_weight_grad(Kin, N, rows):
    rng = np.random.default_rng(Kin + N + rows)
    X = rng.standard_normal((rows, Kin)).astype(np.float32)
    dZ = rng.standard_normal((rows, N)).astype(np.float32)
    out, db = _gemm(2, Kin, N, rows, X, dZ, None)
    ref = X.astype(np.float64).T @ dZ.astype(np.float64)
    mag = np.abs(X.astype(np.float64)).T @ np.abs(dZ.astype(np.float64))
    assert np.all(np.abs(out - ref) <= 1e-5 * mag + 1e-30)
    dbr = dZ.astype(np.float64).sum(0)
    assert np.all(np.abs(db - dbr) <= 1e-5 * np.abs(dZ).astype(np.float64).sum(0) + 1e-30)


@pytest.mark.parametrize("M,N,K", [(300, 512, 512), (257, 86, 512), (100, 256, 49), (70, 512, 1),
                                   (129, 512, 7), (64, 576, 64)])
def test_gemm_dx_bit_exact(M, N, K):
    """dX = dZ W^T is the oracle's linear_bwd chain bit for bit: per element an fmaf chain over
    the K outputs in order from 0 (v_mfma_f32_32x32x2_f32 is a k-ordered fmaf chain), then the
    relu' mask of the layer below"""
    rng = np.random.default_rng(M * 3 + N + K)
    dZ = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)           # W [in = N][out = K]
    H = rng.standard_normal((M, N)).astype(np.float32)
    ref = O.linear_dx(dZ, W)
    out, _ = _gemm(1, M, N, K, dZ, W, None)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    out, _ = _gemm(1, M, N, K, dZ, W, H)
    assert np.array_equal(out, np.where(H > 0, ref, np.float32(0)))


@pytest.mark.parametrize("Kin,N,rows", [(512, 512, 5000), (86, 512, 4099), (256, 8, 3000), (576, 64, 70000),
                                        (64, 8, 31)])
def test_gemm_weight_grad_f64(Kin, N, rows):
    """mode 3 (k_gemm_wg64): every product exact in f64, f64 sums, one rounding to f32 -- the
    f32 rounding of the exact dot product except where the f64 sum's ordering error straddles
    an f32 rounding boundary (~2^-19 of the entries at 10^5 rows): at most one ulp there"""
    rng = np.random.default_rng(Kin * 5 + N + rows)
    X = rng.standard_normal((rows, Kin)).astype(np.float32)
    dZ = rng.standard_normal((rows, N)).astype(np.float32)
    out, db = _gemm(3, Kin, N, rows, X, dZ, None)
    ref = (X.astype(np.float64).T @ dZ.astype(np.float64)).astype(np.float32)
    dbr = dZ.astype(np.float64).sum(0).astype(np.float32)
    for got, want in ((out, ref), (db, dbr)):
        ulps = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
        assert ulps.max() <= 1 and np.count_nonzero(ulps) <= max(2, got.size // 10000), (ulps.max(), np.count_nonzero(ulps))


@pytest.mark.parametrize("Kin,N,rows", [(86, 512, 4099), (256, 8, 3000), (64, 8, 31)])
def test_gemm_weight_grad_row_ordered(Kin, N, rows):
    """mode 4 (k_wg_seq): each entry the f64 sum of the exact products in row order, rounded
    once -- the oracle's linear_bwd loop, so equal to a sequential f64 restatement bit for bit"""
    rng = np.random.default_rng(Kin * 7 + N + rows)
    X = rng.standard_normal((rows, Kin)).astype(np.float32)
    dZ = rng.standard_normal((rows, N)).astype(np.float32)
    out, db = _gemm(4, Kin, N, rows, X, dZ, None)
    acc = np.zeros((Kin, N), np.float64)
    bacc = np.zeros(N, np.float64)
    X64, dZ64 = X.astype(np.float64), dZ.astype(np.float64)
    for r in range(rows):                    # row order, one f64 rounding per addition
        acc += X64[r][:, None] * dZ64[r][None, :]
        bacc += dZ64[r]
    assert np.array_equal(out.view(np.uint32), acc.astype(np.float32).view(np.uint32))
    assert np.array_equal(db.view(np.uint32), bacc.astype(np.float32).view(np.uint32))
