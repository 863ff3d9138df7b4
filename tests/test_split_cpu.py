"""The three-piece bf16 split of variant 4 (csrc/conv_lds.hip split3), restated with numpy on the same bit operations:
h = x with the low 16 bits cleared, r = x - h (fp32), m = r with the low 16 bits cleared, l = r - m.  Checked over
random and edge-case fp32 values: every piece is a bf16 value (low 16 bits zero), h + m + l == x exactly, and every
piece product of two split values is exact in fp32 — the premise of "each fp32 product is formed exactly as the
sum of its 9 piece products" (the GPU side: tests/test_gpu_split.py)."""
import numpy as np

MASK = np.uint32(0xFFFF0000)


def split3(x: np.ndarray):
    xb = x.view(np.uint32)
    h = (xb & MASK).view(np.float32)
    r = (x - h).astype(np.float32)
    m = (r.view(np.uint32) & MASK).view(np.float32)
    l = (r - m).astype(np.float32)
    return h, m, l


def _values():
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2 ** 32, 200_000, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    x = x[np.isfinite(x)]
    # normal range used by training data and weights, plus values with all 24 significant bits set
    y = (rng.standard_normal(100_000) * 10.0 ** rng.uniform(-8, 8, 100_000)).astype(np.float32)
    z = np.array([0.0, -0.0, 1.0, -1.0, np.float32(1) + np.float32(2 ** -23), np.finfo(np.float32).max,
                  np.finfo(np.float32).tiny, 16777215.0, -16777215.0], dtype=np.float32)
    return np.concatenate([x, y, z])


def test_pieces_are_bf16_and_sum_exactly():
    x = _values()
    # ignore values whose remainders fall into the fp32 subnormal range (|x| < 2^-110): bf16 keeps 8 significant
    # bits there only down to 2^-133, the split is exact for every value a training step produces
    x = x[(np.abs(x) > 2.0 ** -100) | (x == 0)]
    h, m, l = split3(x)
    for p in (h, m, l):
        assert not np.any(p.view(np.uint32) & np.uint32(0xFFFF))
    assert np.array_equal(h.astype(np.float64) + m.astype(np.float64) + l.astype(np.float64), x.astype(np.float64))


def test_piece_products_are_exact_in_fp32():
    rng = np.random.default_rng(1)
    a = (rng.standard_normal(50_000) * 10.0 ** rng.uniform(-6, 6, 50_000)).astype(np.float32)
    b = (rng.standard_normal(50_000) * 10.0 ** rng.uniform(-6, 6, 50_000)).astype(np.float32)
    pa, pb = split3(a), split3(b)
    total = np.zeros(a.shape, np.float64)
    for u in pa:
        for v in pb:
            p32 = (u * v).astype(np.float32)
            p64 = u.astype(np.float64) * v.astype(np.float64)
            assert np.array_equal(p32.astype(np.float64), p64)  # 8 x 8 significant bits: no rounding
            total += p64
    assert np.array_equal(total, a.astype(np.float64) * b.astype(np.float64))


def test_sign_flip_of_packed_pieces_negates_exactly():
    """Odd stages / the second wave stage -A by xor-ing the packed pieces' sign bits (0x80008000 per dword)."""
    x = _values()
    x = x[(np.abs(x) > 2.0 ** -100) | (x == 0)]
    for p in split3(x):
        hi = (p.view(np.uint32) >> 16).astype(np.uint32)
        flipped = ((hi ^ np.uint32(0x8000)) << 16).view(np.float32)
        assert np.array_equal(flipped.astype(np.float64), -p.astype(np.float64))
