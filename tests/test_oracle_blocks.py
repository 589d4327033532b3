"""CPU: the block-streamed exact top-k (oracle.search.topk_blocks, used by the full-size GPU parity
tests and bench.py's oracle check) equals the plain f64 oracle (oracle.search.topk)."""
import numpy as np
import pytest

from oracle import search as osearch
from oracle import synth as osynth


def _blocks(x32, sizes):
    r0 = 0
    for b in sizes:
        yield r0, x32[r0:r0 + b]
        r0 += b


@pytest.mark.parametrize("dtype", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("sizes", [[5000], [1, 2047, 2952], [1000, 1000, 1000, 1000, 1000], [4999, 1]])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_topk_blocks_equals_topk(dtype, sizes, k):
    n = sum(sizes)
    stored = osynth.synth_rows(3, 0, n, 256, dtype)
    x64 = osynth.to_f64(stored, dtype).copy()
    q64 = osynth.to_f64(osynth.synth_rows(4, 0, 7, 256, dtype), dtype)
    # planted exact ties (duplicates of query 0's winner) and tombstones (NaN rows)
    top = int(osearch.topk(q64[:1], x64, 1)[1][0, 0])
    for dst in (3, 1999, 4998):
        if dst != top:
            x64[dst] = x64[top]
    x64[[0, 17, 2500]] = np.nan
    ref_s, ref_r = osearch.topk(q64, x64, k)
    got_s, got_r = osearch.topk_blocks(q64, _blocks(x64.astype(np.float32), sizes), k, first_rows=700)
    assert np.array_equal(got_r, ref_r)
    assert np.allclose(got_s, ref_s, rtol=0, atol=1e-12)  # f64 gemm vs gemv summation order


def test_topk_blocks_fewer_rows_than_k():
    x64 = osynth.to_f64(osynth.synth_rows(1, 0, 5, 64, "f32"), "f32").copy()
    x64[2] = np.nan
    q64 = osynth.to_f64(osynth.synth_rows(2, 0, 3, 64, "f32"), "f32")
    ref = osearch.topk(q64, x64, 10)
    got = osearch.topk_blocks(q64, _blocks(x64.astype(np.float32), [2, 3]), 10)
    assert np.array_equal(got[1], ref[1]) and np.allclose(got[0], ref[0], rtol=0, atol=1e-12)
    assert (got[1][:, 4:] == -1).all()


def test_topk_blocks_rejects_inexact_queries():
    with pytest.raises(ValueError):
        osearch.topk_blocks(np.full((1, 4), 0.1), [(0, np.zeros((2, 4), np.float32))], 1)
