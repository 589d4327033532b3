"""CPU: the exact two-pass scan's rule (oracle/screen.py; kernel 10) returns exactly
the brute-force top-k of oracle/search.py, and its quantisation bound is rigorous.

The GPU path is held bit-exact to oracle.screen's int8 copy and to oracle.search's top-k
(tests/test_gpu_screen.py); this file shows on the CPU that the selection rule itself — keep rows
with A >= a_k - e2, re-score exactly — can never lose a row of the true top-k."""
import numpy as np
import pytest

from oracle import screen as oscreen
from oracle import search as osearch
from oracle import synth as osynth


def _corpus(n, d, dtype, seed=5):
    stored = osynth.synth_rows(seed, 0, n, d, dtype)
    return osynth.to_f64(stored, dtype).astype(np.float32)


def _queries(nq, d, dtype, seed=6):
    return osynth.to_f64(osynth.synth_rows(seed, 0, nq, d, dtype), dtype).astype(np.float32)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("d", [768, 1024])
def test_bound_is_rigorous(dtype, d):
    """|exact - s_y A| <= E_q = e2 s_y / 2 for every (query, live row)."""
    x = _corpus(2000, d, dtype)
    y = _queries(16, d, dtype)
    codes, scales, live, stats = oscreen.quantize_tiles(x)
    qc, e2, s = oscreen.quantize_queries(y, stats)
    A = oscreen.screen_scores(codes, scales, qc)[:, :2000].astype(np.float64)
    exact = y.astype(np.float64) @ x.astype(np.float64).T
    err = np.abs(exact - s.astype(np.float64)[:, None] * A)
    bound = e2.astype(np.float64)[:, None] * s.astype(np.float64)[:, None] / 2
    assert (err <= bound).all()
    # and it is not vacuous: the worst case is within a few x of the observed error
    assert bound.max() < 40 * err.max()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("k", [1, 5, 10])
def test_screen_topk_equals_topk(dtype, k):
    n, d = 6000, 768
    x = _corpus(n, d, dtype)
    y = _queries(12, d, dtype)
    # planted exact ties (duplicates of query 0's winner) and tombstones (NaN rows)
    top = int(osearch.topk(y[:1].astype(np.float64), x.astype(np.float64), 1)[1][0, 0])
    for dst in (3, 1999, 4998):
        if dst != top:
            x[dst] = x[top]
    x[[0, 17, 2500]] = np.nan
    s, r, nsv = oscreen.screen_topk(y, x, k)
    rs, rr = osearch.topk(y.astype(np.float64), x.astype(np.float64), k)
    assert np.array_equal(r, rr)
    assert np.allclose(s, rs, atol=1e-12, rtol=0)
    assert (nsv >= k).all() and (nsv < n // 20).all()  # a few % of the rows survive at this size


def test_screen_topk_fewer_live_rows_than_k():
    x = _corpus(40, 768, "bf16")
    x[5:] = np.nan
    y = _queries(3, 768, "bf16")
    s, r, _ = oscreen.screen_topk(y, x, 10)
    rs, rr = osearch.topk(y.astype(np.float64), x.astype(np.float64), 10)
    assert np.array_equal(r, rr) and (r[:, 5:] == -1).all()


def test_quantiser_tiles_and_live_words():
    x = _corpus(70, 768, "bf16")  # 3 tiles, the last holds 6 rows
    x[[1, 33]] = np.nan
    codes, scales, live, stats = oscreen.quantize_tiles(x)
    assert codes.shape == (96, 768) and scales.shape == (3,)
    assert live[0] == 0xFFFFFFFF & ~(1 << 1) and live[1] == 0xFFFFFFFF & ~(1 << 1) and live[2] == 0x3F
    assert (codes[[1, 33]] == 0).all() and (codes[70:] == 0).all()
    assert np.abs(codes).max() == 127
    # reconstruction error per element is at most half a step
    rec = np.repeat(scales, 32)[:70, None].astype(np.float64) * codes[:70]
    ok = ~np.isnan(x).any(axis=1)
    assert (np.abs(x[ok] - rec[ok]) <= np.repeat(scales, 32)[:70][ok, None] / 2 * (1 + 1e-6)).all()
    assert 0.99 < stats[0] < 1.01 and 0 < stats[1] < 0.02


def test_zero_query_keeps_every_row():
    """A zero query scores 0 everywhere: every live row survives (the GPU then takes the fallback)."""
    x = _corpus(100, 768, "bf16")
    y = np.zeros((1, 768), dtype=np.float32)
    s, r, nsv = oscreen.screen_topk(y, x, 5)
    assert nsv[0] == 100 and list(r[0]) == [0, 1, 2, 3, 4]


def test_survivors_cover_the_f32_score_rule():
    """Under the score rule every plan answers with (fl32 of the exact dot desc, row asc): a row whose
    exact score is just below the k-th but rounds to the same f32 and has a smaller row id belongs in the
    answer, so it must survive the cut A >= a_k - e2 (e2 carries two f32 ulps of the k-th score for it,
    ADVICE r4).  Near-ties planted: copies of each query's k-th row with one element moved by one bf16
    step, placed at smaller row ids (exact scores differ by ~1e-9, most round to the same f32)."""
    from oracle import synth as osy
    n, d, k = 4000, 768, 10
    x = _corpus(n, d, "bf16")
    y = _queries(6, d, "bf16")
    ex = y.astype(np.float64) @ x.astype(np.float64).T
    slot = 0
    for i in range(y.shape[0]):
        kth = int(np.lexsort((np.arange(n), -ex[i]))[k - 1])
        for j in range(3):
            v = x[kth].astype(np.float64).copy()
            e = int(np.argsort(np.abs(y[i].astype(np.float64) * v))[j])  # the smallest score change
            # one bf16 step of element e, in the direction that lowers the score a little
            step = np.float64(np.ldexp(1.0, int(np.frexp(abs(v[e]) or 1e-3)[1]) - 8))
            v[e] -= np.sign(y[i, e] or 1.0) * step
            x[slot] = osy.bf16_bits_to_f32(osy.f32_to_bf16_bits(v.astype(np.float32)))
            slot += 1
    codes, scales, live, stats = oscreen.quantize_tiles(x)
    qc, e2, _ = oscreen.quantize_queries(y, stats)
    A = oscreen.screen_scores(codes, scales, qc)[:, :n]
    ex = y.astype(np.float64) @ x.astype(np.float64).T
    ties = 0
    for i in range(y.shape[0]):
        f32 = ex[i].astype(np.float32)
        order = np.lexsort((np.arange(n), -f32))  # the score rule, on all rows
        fk = f32[order[k - 1]]
        want = np.nonzero(f32 >= fk)[0]  # every row the rule could place in the top k
        ties += int(np.sum(f32 == fk)) - 1
        ak = np.partition(A[i], n - k)[n - k]
        t = np.float32(ak - e2[i])
        assert (A[i, want] >= t).all()
    assert ties >= 1  # the planted near-ties exist in f32
