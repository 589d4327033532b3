"""Kernel 10's XCD-balanced tile split (k_scan_screen.h, `bal` branch), restated on the host: for any
weights the quantiser can hand it (integers in [512, 2048]) the blocks' tile sets are disjoint and cover
every tile exactly once, and with >= 64 tiles per block on average every block keeps >= 2 tiles (so no
block returns before writing its lists).  Host logic only; the GPU side is checked end to end by
tests/test_gpu_fullsize.py and tests/test_gpu_screen.py."""
import numpy as np
import pytest


def block_tiles(ntiles, nblk, w, b):
    """The tiles block b takes: the kernel's integer arithmetic, line for line."""
    xc, j, bpx = b & 7, b >> 3, nblk >> 3
    pre = sum(int(w[x]) for x in range(xc))
    tot = sum(int(v) for v in w)
    t_lo = ntiles * pre // tot
    t_hi = ntiles * (pre + int(w[xc])) // tot
    tb0 = t_lo + j
    nt = (t_hi - tb0 + bpx - 1) // bpx if tb0 < t_hi else 0
    return [tb0 + i * bpx for i in range(nt)]


@pytest.mark.parametrize("ntiles", [64 * 256, 39063, 312500, 390625])
def test_split_is_a_partition(ntiles):
    rng = np.random.default_rng(ntiles)
    nblk = 256
    for trial in range(20):
        w = rng.integers(512, 2049, size=8) if trial else np.full(8, 1024)
        if trial == 1:
            w = np.array([512, 2048, 512, 2048, 512, 2048, 512, 2048])
        if trial == 2:
            w = np.array([512] + [2048] * 7)
        seen = np.zeros(ntiles, dtype=np.int32)
        counts = []
        for b in range(nblk):
            t = block_tiles(ntiles, nblk, w, b)
            counts.append(len(t))
            seen[t] += 1
        assert (seen == 1).all()
        assert min(counts) >= 2


def test_equal_weights_balance_the_xcds():
    ntiles, nblk = 312500, 256
    per_xcd = [sum(len(block_tiles(ntiles, nblk, [1024] * 8, b)) for b in range(x, nblk, 8)) for x in range(8)]
    assert max(per_xcd) - min(per_xcd) <= 1
