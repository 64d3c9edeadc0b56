"""Host restatements of two index maps the round-6 kernels rely on for
correctness (CPU only; the GPU suite checks their results bitwise):
  - xcd_window_block (csrc/knn.hip): the windowed XCD swizzle of the gather's
    walk blocks must be a bijection on the launch's walk blocks, whatever the
    grid size, the window size k and the number of retry blocks in front;
  - the local selection finish's histogram bin (csrc/kdtree.hip,
    k_kd_local_sel): bin(key) = min(nb - 1, (uint)((float)(key - lo) * scale))
    with scale = nb / ((float)(hi - lo) + 1) must be monotone non-decreasing in
    the key and inside [0, nb), so that equal keys share a bin and the bins
    follow the order (the rank of the median is then found bin by bin)."""
import numpy as np
import pytest


def xcd_window_block(f: int, bid: int, grid: int, k: int) -> int:
    """csrc/knn.hip xcd_window_block<k>(f, bid) with gridDim.x = grid."""
    if k == 0:
        return f
    w = 8 * k
    nb = grid - (bid - f)
    if f >= nb - nb % w:
        return f
    return (f - f % w) + (bid % 8) * k + (f % w) // 8


@pytest.mark.parametrize("k", [0, 1, 4, 16, 32, 128])
@pytest.mark.parametrize("nwalk,nrb", [(1, 0), (7, 0), (255, 0), (256, 3), (1000, 0), (1024, 5), (4097, 17),
                                       (8 * 32 * 3 + 11, 0), (141_000, 7057)])
def test_xcd_window_block_is_a_bijection(k, nwalk, nrb):
    grid = nrb + nwalk
    got = [xcd_window_block(b - nrb, b, grid, k) for b in range(nrb, grid)]
    assert sorted(got) == list(range(nwalk))


def test_xcd_window_block_groups_by_label():
    """inside a full window the blocks of one XCD label take k consecutive pieces"""
    k, nrb, grid = 32, 3, 3 + 8 * 32 * 4
    for w in range(4):
        for label in range(8):
            pieces = sorted(xcd_window_block(b - nrb, b, grid, k) for b in range(nrb + w * 256, nrb + (w + 1) * 256)
                            if b % 8 == label)
            assert pieces == list(range(pieces[0], pieces[0] + k)), (w, label)


def bins(keys, lo, hi, nb):
    scale = np.float32(nb) / (np.float32(hi - lo) + np.float32(1.0))
    x = (keys - np.uint32(lo)).astype(np.float32) * scale
    return np.minimum(np.uint32(nb - 1), x.astype(np.uint32))


@pytest.mark.parametrize("nb", [1024, 512, 256, 128])
def test_local_select_bins_monotone(nb):
    rng = np.random.default_rng(11)
    for trial in range(200):
        # key ranges from one key to the full 32-bit range, clustered keys
        lo = int(rng.integers(0, 2**32 - 1))
        span = int(rng.choice([0, 1, 2, 7, 1000, 2**20, 2**31, 2**32 - 1 - lo]))
        hi = min(2**32 - 1, lo + span)
        keys = np.sort(rng.integers(lo, hi + 1, size=700, dtype=np.uint64).astype(np.uint32))
        keys = np.concatenate([keys, np.array([lo, hi], np.uint32)])
        keys.sort()
        b = bins(keys, lo, hi, nb)
        assert b.max() < nb and b.min() >= 0
        assert np.all(np.diff(b.astype(np.int64)) >= 0), (lo, hi)   # monotone: equal keys share a bin
