"""Model of the config-4 tile plan's merge-path split (csrc/tile.hip,
tile_split_kernel): a tile after its document's previous tile gallops from a
proportional guess inside the window its predecessor's split bounds
(merge_path_gallop) instead of bisecting the whole diagonal (merge_path_in).
This restates both searches line by line and checks that they agree at every
tile boundary of random sorted runs, dst first on equal keys (awset.go:107-161's
merge order, the same rule the oracle's join uses).  CPU only."""
import random

import pytest


def _p(dk, sk, k, i):  # split > i
    return dk[i] <= sk[k - 1 - i]


def merge_path_in(dk, sk, k, lo, hi):
    while lo < hi:
        mid = (lo + hi) >> 1
        if _p(dk, sk, k, mid):
            lo = mid + 1
        else:
            hi = mid
    return lo


def merge_path_gallop(dk, sk, k, lo, hi, g):
    if lo >= hi:
        return lo
    g = min(max(g, lo), hi - 1)
    if _p(dk, sk, k, g):
        lo = g + 1
        step = 1
        while g + step < hi:
            j = g + step
            if not _p(dk, sk, k, j):
                hi = j
                break
            lo = j + 1
            step <<= 1
    else:
        hi = g
        step = 1
        while step <= g - lo:
            j = g - step
            if _p(dk, sk, k, j):
                lo = j + 1
                break
            hi = j
            step <<= 1
    return merge_path_in(dk, sk, k, lo, hi)


@pytest.mark.parametrize("seed", range(6))
def test_gallop_matches_bisection(seed):
    rng = random.Random(seed)
    for _ in range(60):
        nd, ns = rng.randint(0, 2500), rng.randint(0, 2500)
        span = rng.choice([nd + ns + 5, 3 * (nd + ns) + 5, 40])  # 40: many equal keys across the runs
        dk = sorted(rng.choice(range(span)) if span == 40 else v for v in rng.sample(range(span + nd + ns), nd))
        sk = sorted(rng.choice(range(span)) if span == 40 else v for v in rng.sample(range(span + nd + ns), ns))
        tile = rng.choice([1, 7, 64, 1024])
        prev = None
        for t in range(max(1, -(-(nd + ns) // tile))):
            k = min(t * tile, nd + ns)
            lo, hi = max(0, k - ns), min(k, nd)
            full = merge_path_in(dk, sk, k, lo, hi)
            # a run's first tile: from the proportional point of the whole diagonal
            assert merge_path_gallop(dk, sk, k, lo, hi, (k * nd) // max(nd + ns, 1)) == full
            if prev is not None:  # the kernel's windowed call for tile t after tile t-1
                g = prev + (tile * nd) // max(nd + ns, 1)
                got = merge_path_gallop(dk, sk, k, max(lo, prev), min(hi, prev + tile), g)
                assert got == full, (nd, ns, tile, t)
            prev = full
