"""CPU: the closed form of cr_math.h inv_len_unit (1/sqrt(l2) for l2 within 1024 ulps of 1.0) equals
the correctly rounded 1.0f / sqrtf(l2) over its whole window, and the window is inside the range
where the form holds.  The same comparison runs on the GPU over [2^-100, 2^100]
(tests/hip/crmath_check.hip)."""
import numpy as np


def _closed_form(d):
    j = (-d + 1) >> 1
    return np.where(d >= 0, 0x3F800000 - (d & ~1), 0x3F800000 + ((j + 1) >> 1))


def _reference(d):
    x = (0x3F800000 + d).astype(np.uint32).view(np.float32)
    return (np.float32(1.0) / np.sqrt(x)).view(np.uint32).astype(np.int64)


def test_inv_len_unit_window_exact():
    d = np.arange(-1024, 1025, dtype=np.int64)
    assert np.array_equal(_closed_form(d), _reference(d))


def test_inv_len_unit_margin():
    """The form holds well beyond the window used (first failure past +2897 ulps)."""
    d = np.arange(-2897, 2898, dtype=np.int64)
    assert np.array_equal(_closed_form(d), _reference(d))
    d = np.arange(2898, 4096, dtype=np.int64)
    assert not np.array_equal(_closed_form(d), _reference(d))


def _masked_form(d):
    """inv_len_unit_cf on the bits b of l2: 0x7F000000 - (b & ~1) for b >= 1.0, else
    0x3F800000 + ((0x3F800003 - b) >> 2), in uint32 arithmetic."""
    b = (np.int64(0x3F800000) + d).astype(np.uint32)
    up = np.uint32(0x7F000000) - (b & np.uint32(0xFFFFFFFE))
    dn = np.uint32(0x3F800000) + ((np.uint32(0x3F800003) - b) >> np.uint32(2))
    return np.where(b.astype(np.int32) >= 0x3F800000, up, dn).astype(np.int64)


def test_inv_len_unit_cf_equals_closed_form():
    d = np.arange(-2897, 2898, dtype=np.int64)
    assert np.array_equal(_masked_form(d), _closed_form(d))


def _normalize(v):
    """glm::normalize in float32 as the device evaluates it: v * (1 / sqrt(dot(v, v))), each op rounded."""
    v = v.astype(np.float32)
    l2 = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    s = np.float32(1.0) / np.sqrt(l2)
    return v * s[:, None]


def test_normalized_vectors_stay_in_the_window():
    """renormalized_again() drops inv_len_unit's range test: a vector that came out of a normalization
    has its squared length within a few ulps of 1 (here <= 8 over 4M random directions of all scales,
    normalized once and twice), far inside the +-1024-ulp window of the closed form."""
    g = np.random.default_rng(7)
    v = g.normal(size=(1 << 22, 3)) * np.exp(g.uniform(-20, 20, size=(1 << 22, 1)))
    for _ in range(2):
        v = _normalize(v)
        l2 = ((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]).astype(np.float32)
        d = l2.view(np.int32).astype(np.int64) - 0x3F800000
        assert np.abs(d).max() <= 8, np.abs(d).max()
