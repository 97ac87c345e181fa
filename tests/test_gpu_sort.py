"""The LBVH build's hand-written device primitives (csrc/kernels_sort.hip) against numpy, bit for bit.

`radix_sort_pairs_u64` is an 8-pass LSD radix sort that claims stability element for element (the
Morton keys of the build, 63 bits, value = reference id); `scan_u32` an exclusive prefix sum in
4096-count tiles with a single-workgroup pass over the tile sums.  They replace the rocPRIM calls
of r01-r03 and the Embree build (/root/reference/src/backends/EmbreeBackend.cpp:82-181).  Sizes
cover n = 0, a partial first tile, exact tiles, one past a tile, many tiles, more than one 4096-tile
level of tile sums (the sort's histogram scan at 10M keys has 256 x 2442 counts), heavy duplicates
(stability), and the full 64-bit key range.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 255, 4095, 4096, 4097, 1_000_003, 10_000_008]


def _keys(n, kind, rng):
    if kind == "full":  # every bit of the 64-bit key
        return rng.integers(0, np.iinfo(np.uint64).max, n, dtype=np.uint64, endpoint=True)
    if kind == "dup":  # heavy duplicates: 37 distinct keys spread over all 8 digit positions
        pool = rng.integers(0, np.iinfo(np.uint64).max, 37, dtype=np.uint64, endpoint=True)
        return pool[rng.integers(0, 37, n)]
    # morton: 63-bit codes as k_morton makes them, sorted input order with runs (the build's case)
    return rng.integers(0, 1 << 63, n, dtype=np.uint64)


# every size with every key kind, except the 10M case once (morton keys: the build's own)
CASES = [(n, kind) for n in SIZES for kind in ("full", "dup", "morton") if n < 10_000_000 or kind == "morton"]


@pytest.mark.parametrize("n,kind", CASES)
def test_radix_sort_pairs_matches_stable_argsort(renderer, n, kind):
    rng = np.random.default_rng(n * 7 + len(kind))
    keys = _keys(n, kind, rng)
    vals = np.arange(n, dtype=np.uint32) ^ np.uint32(0x5A5A5A5A)  # distinct values: order is observable
    ko, vo = renderer.sort_pairs_u64(keys, vals)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ko, keys[order])
    assert np.array_equal(vo, vals[order])  # stability: equal keys keep their input order


@pytest.mark.parametrize("n", SIZES + [4096 * 4097 + 5])
def test_scan_u32_matches_cumsum(renderer, n):
    rng = np.random.default_rng(n + 3)
    counts = rng.integers(0, 1 << 12, n, dtype=np.uint32)
    if n > 16:
        counts[:: max(1, n // 17)] = np.uint32(0xFFFFFFF0)  # large counts: the sum wraps mod 2^32 as uint32 does
    out = renderer.scan_u32(counts)
    ref = (np.cumsum(counts, dtype=np.uint64) - counts.astype(np.uint64)).astype(np.uint32)
    assert np.array_equal(out, ref)


def test_scan_u32_in_bounds_of_the_sort_histograms(renderer):
    # the radix sort's histogram scan: 256 digits x tiles counts, each <= 4096
    tiles = 2442
    counts = np.random.default_rng(5).integers(0, 4097, 256 * tiles, dtype=np.uint32)
    out = renderer.scan_u32(counts)
    assert out[0] == 0 and np.array_equal(out[1:], np.cumsum(counts, dtype=np.uint64)[:-1].astype(np.uint32))
