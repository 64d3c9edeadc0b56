"""Host restatements of two index maps the round-6 kernels rely on for
correctness (CPU only; the GPU suite checks their results bitwise):
  - xcd_window_block (csrc/knn.hip): the windowed XCD swizzle of the gather's
    walk blocks must be a bijection on the launch's walk blocks, whatever the
    grid size, the window size k and the number of retry blocks in front;
  - the local selection finish's histogram bin (csrc/kdtree.hip,
    k_kd_local_sel): bin(key) = min(nb - 1, (uint)((float)(key - lo) * scale))
    with scale = nb / ((float)(hi - lo) + 1) must be monotone non-decreasing in
    the key and inside [0, nb), so that equal keys share a bin and the bins
    follow the order (the rank of the median is then found bin by bin);
  - the guessed follower cut-offs (csrc/knn.hip, seed_bounds): the guess is
    never looser than the guaranteed bound; and k_gather_fmark's retry list:
    every flagged follower exactly once, written downwards from entry nq - 1
    without reaching the leaders' range, each block's ranks in walk order."""
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


# ---- guessed follower cut-offs (csrc/knn.hip, seed_bounds / k_gather_fmark)

def seed_bounds(lead_w, lead_pos, q, alpha=0.25, beta=0.1):
    """knn.hip seed_bounds: (guaranteed, guessed) squared bounds, f64."""
    d = np.sqrt(((q - lead_pos) ** 2).sum(-1))
    rl = np.sqrt(lead_w)
    c = rl + d
    sq = lambda x: x * x * (1.0 + 1e-5) + 1e-30
    return sq(c * (1.0 + 1e-6)), sq(np.minimum(c, rl * (1.0 + beta) + alpha * d) * (1.0 + 1e-6))


def test_guess_never_looser_than_guarantee():
    rng = np.random.default_rng(5)
    for alpha, beta in ((0.25, 0.1), (0.0, 0.0), (0.0, 0.3), (1.0, 0.0), (0.5, 2.0)):
        w = rng.uniform(0, 4, 10000) ** 2
        g, e = seed_bounds(w, rng.normal(size=(10000, 3)), rng.normal(size=(10000, 3)), alpha, beta)
        assert np.all(e <= g)
    # alpha = 1, beta = 0 is the guaranteed bound itself
    w = rng.uniform(0, 4, 1000) ** 2
    g, e = seed_bounds(w, rng.normal(size=(1000, 3)), rng.normal(size=(1000, 3)), 1.0, 0.0)
    assert np.array_equal(g, e)


def fmark(flags, nl, grid, per=64, block=256):
    """k_gather_fmark restated: blocks of block * per flags in a grid-stride
    loop, blocks served in an arbitrary order (the atomic), each writing its
    flagged ranks in order downwards from nq - 1."""
    nq = len(flags)
    retry = np.full(nq, -1, np.int64)
    chunks = list(range(0, nq, block * per))
    order = np.random.default_rng(len(flags)).permutation(len(chunks))
    cnt = 0
    for c in order:
        r0 = chunks[c]
        ranks = [r for r in range(r0, min(nq, r0 + block * per)) if flags[r]]
        for k, r in enumerate(ranks):
            retry[nq - 1 - (cnt + k)] = r
        cnt += len(ranks)
    return retry, cnt


@pytest.mark.parametrize("nq,p", [(1, 1.0), (100, 0.5), (20000, 0.01), (70001, 0.003), (70001, 0.0)])
def test_follower_retry_list_layout(nq, p):
    rng = np.random.default_rng(nq)
    s = 20
    nl = (nq + s - 1) // s
    flags = np.zeros(nq, bool)
    followers = np.array([r for r in range(nq) if r % s], np.int64)
    if len(followers):
        flags[followers[rng.random(len(followers)) < p]] = True
    retry, cnt = fmark(flags, nl, grid=8)
    assert cnt == flags.sum() and cnt <= nq - nl          # the leaders' range [0, nl) is never reached
    lst = retry[nq - cnt:][::-1]                          # written downwards from nq - 1
    assert sorted(lst.tolist()) == np.nonzero(flags)[0].tolist()
    chunk = 256 * 64
    for c in np.unique(lst // chunk):                     # each block's ranks contiguous and in walk order
        pos = np.nonzero(lst // chunk == c)[0]
        assert np.all(np.diff(pos) == 1) and np.all(np.diff(lst[pos]) > 0)
