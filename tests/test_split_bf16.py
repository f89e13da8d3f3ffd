"""The split-bf16 arithmetic of the minibatch kernel (k_update.hip k_minibatch_split):
every f32 operand x is split exactly into three bf16 pieces x = x0 + x1 + x2 (each
rounded to nearest even, as v_cvt_pk_bf16_f32 does), and a product x*y is taken as the
six piece products of order <= 2 (x0y0, x0y1, x1y0, x0y2, x1y1, x2y0), each exact in
f32, accumulated in f32.  Host emulation (numpy, no GPU): the split is exact for normal
f32 values; |x1| <= 2^-8 |x| and |x2| <= 2^-16 |x|, so each dropped product (x1y2, x2y1,
x2y2) is at most 2^-24 |xy| and the three together at most (2^-23 + 2^-32) |xy|; with the
f32 additions the six-product sum is within 2^-22 of the true product.  The hardware's
own accumulation is checked on the GPU against the oracle (tests/test_gpu_split_kernel.py)."""
import numpy as np


def bf16_rne(x):
    """f32 -> nearest bf16 (ties to even), returned as f32"""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    x = np.asarray(x, np.float32)
    a = bf16_rne(x)
    r = (x - a).astype(np.float32)
    b = bf16_rne(r)
    c = bf16_rne((r - b).astype(np.float32))
    return a, b, c


def test_split_is_exact():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-30, 30, 200000))).astype(np.float32)
    a, b, c = split3(x)
    assert np.array_equal(((a + b).astype(np.float32) + c).astype(np.float32), x)
    # each piece carries at most 8 significant bits
    for p in (a, b, c):
        assert np.all((p.view(np.uint32) & 0xFFFF) == 0)


def test_six_products_match_f32_multiply():
    rng = np.random.default_rng(1)
    n = 200000
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    xa, xb, xc = split3(x)
    ya, yb, yc = split3(y)
    # the piece products are exact in f32 (8 x 8 significant bits); the kernel adds them in f32
    terms = [xc * ya, xb * yb, xa * yc, xb * ya, xa * yb, xa * ya]
    # the dropped products, in f64 (exact): the stated bound
    ax, ay = np.abs(x.astype(np.float64)), np.abs(y.astype(np.float64))
    assert np.all(np.abs(xb.astype(np.float64)) <= 2.0 ** -8 * ax)
    assert np.all(np.abs(xc.astype(np.float64)) <= 2.0 ** -16 * ax)
    dropped = (np.abs(xb.astype(np.float64) * yc) + np.abs(xc.astype(np.float64) * yb)
               + np.abs(xc.astype(np.float64) * yc))
    assert np.all(dropped <= (2.0 ** -23 + 2.0 ** -32) * ax * ay)
    s = np.zeros(n, np.float32)
    for t in terms:
        s = (s + t.astype(np.float32)).astype(np.float32)
    exact = x.astype(np.float64) * y.astype(np.float64)
    rel = np.abs(s.astype(np.float64) - exact) / np.abs(exact)
    f32 = np.abs((x * y).astype(np.float64) - exact) / np.abs(exact)
    assert rel.max() < 2.0 ** -22
    assert np.median(rel) <= 2.0 * np.median(f32) + 1e-12
