"""CPU check of the arithmetic behind the split-bf16 ("x6") contractions
(msp_conv_x6.hip): every fp32 value is written exactly as three
bf16 pieces (round-to-nearest-even, residuals formed in fp32), and the six
piece products with i + j <= 2 reproduce w*x to about one fp32 rounding.

The bf16 rounding here restates v_cvt_pk_bf16_f32 (RNE on the upper 16 bits);
the GPU kernels themselves are checked against fp64 in
tests/test_gpu_ops.py::test_conv_tile_split_bf16_accuracy."""
import numpy as np


def bf16_rne(v):
    """fp32 -> nearest bf16 (ties to even), returned as fp32."""
    u = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def split3(v):
    v = np.asarray(v, dtype=np.float32)
    p0 = bf16_rne(v)
    r1 = (v - p0).astype(np.float32)  # exact in fp32
    p1 = bf16_rne(r1)
    r2 = (r1 - p1).astype(np.float32)  # exact in fp32
    p2 = bf16_rne(r2)
    return p0, p1, p2


def _values(n, seed):
    rng = np.random.default_rng(seed)
    mant = rng.uniform(1.0, 2.0, n)
    expo = rng.integers(-60, 60, n)
    sign = rng.choice([-1.0, 1.0], n)
    return (sign * mant * np.exp2(expo)).astype(np.float32)


def test_three_piece_split_is_exact():
    v = np.concatenate([_values(200000, 0), np.float32([0.0, -0.0, 1.0, -1.5, 3.0e-30, 7.0e30])])
    p0, p1, p2 = split3(v)
    # the last piece carries at most 8 significant bits, so it is exactly a bf16
    assert np.array_equal(bf16_rne(p2), p2)
    recon = p0.astype(np.float64) + p1.astype(np.float64) + p2.astype(np.float64)
    assert np.array_equal(recon, v.astype(np.float64))
    a = np.abs(v.astype(np.float64))
    assert np.all(np.abs(p1) <= 2.0 ** -8 * a + 0.0)
    assert np.all(np.abs(p2) <= 2.0 ** -16 * a + 0.0)


def test_six_products_error_is_one_fp32_rounding():
    w, x = _values(200000, 1), _values(200000, 2)
    w0, w1, w2 = (p.astype(np.float64) for p in split3(w))
    x0, x1, x2 = (p.astype(np.float64) for p in split3(x))
    six = w2 * x0 + w1 * x1 + w0 * x2 + w1 * x0 + w0 * x1 + w0 * x0  # each product exact in fp64
    exact = w.astype(np.float64) * x.astype(np.float64)
    rel = np.abs(six - exact) / np.abs(exact)
    assert rel.max() <= 2.0 ** -23
    # an fp32 fmaf of the same product rounds once: 2^-24 relative at most
    f32 = (w * x).astype(np.float64)
    assert (np.abs(f32 - exact) / np.abs(exact)).max() <= 2.0 ** -24


def test_dot_product_error_matches_fp32_class():
    """A 27 x 64-term contraction (one output of a level-1 conv) through the six
    piece products, accumulated in fp32 in product order, against fp64: the
    error stays within a small multiple of the plain fp32 dot product's."""
    rng = np.random.default_rng(3)
    worst_x6, worst_f32 = 0.0, 0.0
    for _ in range(200):
        w = (rng.standard_normal(27 * 64) / 40.0).astype(np.float32)
        x = rng.standard_normal(27 * 64).astype(np.float32)
        w0, w1, w2 = split3(w)
        x0, x1, x2 = split3(x)
        acc = np.float32(0.0)
        for a, b in ((w2, x0), (w1, x1), (w0, x2), (w1, x0), (w0, x1), (w0, x0)):
            acc = np.float32(acc + np.float32(np.dot(a.astype(np.float64), b.astype(np.float64))))
        acc32 = np.float32(0.0)
        for i in range(0, w.size, 32):
            acc32 = np.float32(acc32 + np.float32(np.dot(w[i:i + 32].astype(np.float64),
                                                         x[i:i + 32].astype(np.float64))))
        ref = np.dot(w.astype(np.float64), x.astype(np.float64))
        scale = np.abs(w.astype(np.float64) * x).sum()
        worst_x6 = max(worst_x6, abs(float(acc) - ref) / scale)
        worst_f32 = max(worst_f32, abs(float(acc32) - ref) / scale)
    assert worst_x6 <= 4.0 * worst_f32 + 2.0 ** -24, (worst_x6, worst_f32)
