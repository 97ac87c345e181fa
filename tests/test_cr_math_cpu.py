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
