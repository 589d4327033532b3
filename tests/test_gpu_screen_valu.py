"""GPU: kernel 11 (k_screen_valu.hip) — the exact two-pass scan of a few questions
(nq <= 8, 5 <= k <= 16) in one launch over the index's int8 copy, with the gated exact one-launch
search behind it.  Config 2 (100k x 768 f32, nq 1, k 10) is this path.

Bars (as tests/test_gpu_screen.py): the f32 int8 copy is BIT-EXACT with oracle/screen.py; every
search returns oracle/search.py's brute-force top-k under check_topk (rows identical outside the
2e-6 tie band, no duplicates, scores within 1e-5 of the f64 score); the forced fallback (screen
mode 2) and the exact scan (screen off) return the same rows."""
import numpy as np
import pytest
import torch

from oracle import screen as oscreen
from oracle import search as osearch
from oracle import synth as osynth

pytestmark = pytest.mark.gpu

TOL, TIE = 1e-5, 2e-6


@pytest.fixture(scope="module")
def rindex():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import rfx.index as ri
    return ri


def _widen(stored, dtype):
    return osynth.to_f64(stored, dtype).astype(np.float32)


def _make(rindex, n, d, dtype, seed=31, screen=1):
    ix = rindex.DeviceIndex(d, dtype)
    ix.add_synthetic(seed, n)
    if screen:
        ix.enable_screen(screen)
    return ix, _widen(osynth.synth_rows(seed, 0, n, d, dtype), dtype)


def _queries(rindex, nq, d, dtype, seed=32):
    return rindex.synth_rows(seed, 0, nq, d, dtype), _widen(osynth.synth_rows(seed, 0, nq, d, dtype), dtype)


def _check(ix, rows32, q, q32, k, row_mask=None, allowed=None):
    s, r = ix.search(q, k, row_mask=row_mask)
    torch.cuda.synchronize()
    s, r = s.cpu().numpy(), r.cpu().numpy()
    rows64 = rows32.astype(np.float64)
    if allowed is not None:
        rows64 = rows64.copy()
        rows64[~allowed] = np.nan
    q64 = q32.astype(np.float64)
    ref_s, ref_r = osearch.topk(q64, rows64, k)
    probs = osearch.check_topk(s, r, ref_s, ref_r, lambda qi, rr: rows64[rr] @ q64[qi], tol=TOL, tie_band=TIE)
    assert not probs, probs[:5]
    return s, r


def test_f32_int8_copy_bit_exact(rindex):
    n = 4000 + 9
    ix, rows32 = _make(rindex, n, 768, "f32")
    ix.tombstone([5, 100, 4008])
    rows32[[5, 100, 4008]] = np.nan
    codes, scales, live, stats = ix.screen_read(0, (n + 31) // 32)
    rc, rs, rl, rst = oscreen.quantize_tiles(rows32)
    assert codes.tobytes() == rc.tobytes() and scales.tobytes() == rs.tobytes() and live.tobytes() == rl.tobytes()
    assert np.allclose(stats[:2], rst[:2], rtol=2e-7, atol=0) and stats[2] == rst[2]


@pytest.mark.parametrize("dtype,d", [("f32", 768), ("bf16", 768), ("f16", 768), ("f32", 1024), ("bf16", 1024)])
@pytest.mark.parametrize("nq,k", [(1, 10), (2, 10), (3, 5), (4, 12), (8, 16)])
def test_kernel11_matches_oracle(rindex, dtype, d, nq, k):
    ix, rows32 = _make(rindex, 30000, d, dtype)
    assert ix.search_plan(nq, k) == 11
    q, q32 = _queries(rindex, nq, d, dtype)
    _check(ix, rows32, q, q32, k)


def test_config2_shape(rindex):
    """BASELINE configs[1]: 100k x 768 f32, one query, k 10 — 20 different lone questions."""
    ix, rows32 = _make(rindex, 100_000, 768, "f32")
    q, q32 = _queries(rindex, 20, 768, "f32", seed=1)
    for i in range(20):
        _check(ix, rows32, q[i:i + 1].contiguous(), q32[i:i + 1], 10)


@pytest.mark.parametrize("dtype,nq,k", [("f32", 1, 10), ("f32", 8, 10), ("bf16", 3, 16)])
def test_kernel11_list_path_larger_store(rindex, dtype, nq, k):
    """More than 128 rows per wave (200k rows, ~200 per wave): the waves keep their first two 64-row chunks'
    scores, select and sort their 16 best, and insert the later chunks into those sorted lists (round 6);
    ties at the kept set's edge included (duplicated rows)."""
    ix, rows32 = _make(rindex, 200_000, 768, dtype)
    assert ix.search_plan(nq, k) == 11
    q, q32 = _queries(rindex, nq, 768, dtype, seed=7)
    _check(ix, rows32, q, q32, k)
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    ix.add(ix.read(top, 1).repeat(30, 1))  # 30 copies of query 0's winner: ties at every wave's 16th
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 30, axis=0)])
    _check(ix, rows32, q, q32, k)
    ix.close()


def test_kernel11_fallback_and_exact_agree(rindex):
    ix, rows32 = _make(rindex, 40000, 768, "f32")
    q, q32 = _queries(rindex, 4, 768, "f32")
    s1, r1 = _check(ix, rows32, q, q32, 10)
    ix.enable_screen(2)  # the screen declines every batch: the gated exact search answers
    s2, r2 = _check(ix, rows32, q, q32, 10)
    ix.enable_screen(0)
    assert ix.search_plan(4, 10) == 0
    s3, r3 = _check(ix, rows32, q, q32, 10)
    assert np.array_equal(r1, r3) and np.array_equal(r2, r3)
    # the state left behind by a fallback does not leak into the next screened search
    ix.enable_screen(1)
    s4, r4 = _check(ix, rows32, q, q32, 10)
    assert np.array_equal(r4, r3)


def test_kernel11_duplicates_tombstones_masks(rindex):
    ix, rows32 = _make(rindex, 20000, 768, "bf16", screen=0)
    q, q32 = _queries(rindex, 2, 768, "bf16")
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    # 40 copies of query 0's winner: more than a wave list holds -> dropped rows at the bound -> fallback
    first = ix.add(ix.read(top, 1).repeat(40, 1))
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 40, axis=0)])
    ix.enable_screen(1)
    s, r = _check(ix, rows32, q, q32, 16)
    assert r[0, 0] == top and list(r[0, 1:16]) == list(range(first, first + 15))
    dead = [top, first + 3, 777]
    ix.tombstone(dead)
    rows32[dead] = np.nan
    _check(ix, rows32, q, q32, 10)
    rng = np.random.default_rng(5)
    allowed = rng.random(rows32.shape[0]) < 0.25
    words = np.zeros((rows32.shape[0] + 31) // 32, dtype=np.uint32)
    for i in np.nonzero(allowed)[0]:
        words[i >> 5] |= np.uint32(1 << (i & 31))
    m = torch.from_numpy(words.view(np.int32)).cuda()
    _check(ix, rows32, q, q32, 10, row_mask=m, allowed=allowed & ~np.isnan(rows32[:, 0]))


def test_kernel11_small_stores(rindex):
    for n in (3, 17, 100, 700):  # fewer rows than k, sub-tile, a few waves
        ix, rows32 = _make(rindex, n, 768, "f32", seed=40 + n)
        q, q32 = _queries(rindex, 1, 768, "f32")
        s, r = _check(ix, rows32, q, q32, 10)
        if n < 10:
            assert (r[0, n:] == -1).all()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_kernel11_lone_question_fallback_in_launch(rindex, dtype):
    """A lone question runs the exact fallback INSIDE kernel 11's launch (round 5: workgroups claim
    virtual blocks of the one-launch VALU search): forced (screen mode 2) and natural (40 copies of the
    winner, more than a wave list holds), each equal to the exact scan; the state a fallback leaves does
    not leak into the next screened search."""
    ix, rows32 = _make(rindex, 60000, 768, dtype, screen=0)
    q, q32 = _queries(rindex, 3, 768, dtype)
    exact = [_check(ix, rows32, q[i:i + 1].contiguous(), q32[i:i + 1], 10) for i in range(3)]
    for mode in (2, 1, 2, 1):
        ix.enable_screen(mode)
        assert ix.search_plan(1, 10) == 11
        for i in range(3):
            s, r = _check(ix, rows32, q[i:i + 1].contiguous(), q32[i:i + 1], 10)
            assert np.array_equal(r, exact[i][1]) and np.array_equal(s, exact[i][0])
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    ix.enable_screen(0)
    first = ix.add(ix.read(top, 1).repeat(40, 1))
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 40, axis=0)])
    ix.enable_screen(1)
    s, r = _check(ix, rows32, q[:1].contiguous(), q32[:1], 16)
    assert r[0, 0] == top and list(r[0, 1:16]) == list(range(first, first + 15))


@pytest.mark.parametrize("unordered", [False, True])
def test_kernel11_from_two_streams_at_once(rindex, monkeypatch, unordered):
    """Kernel 11 issued from two streams of one device at once: a store sharded over four logical shards
    of this GPU (each shard's search on its own stream) plus a second store on a third stream, lone
    questions, the screen forced to decline half the time (the in-launch fallback runs while other
    kernel-11 launches are in flight).  librfx orders kernel-11 launches per device; with that ordering
    switched off (RFX_K11_UNORDERED=1) launches overlap and waiting blocks may give up, and the answers
    must still be the oracle's."""
    from rfx.sharded import ShardedIndex
    if unordered:
        monkeypatch.setenv("RFX_K11_UNORDERED", "1")
    n = 120_000
    sh = ShardedIndex(768, "f32", [0, 0, 0, 0])
    cuts = sh._cuts(n)
    for i, s in enumerate(sh.shards):
        s.add_synthetic(51, cuts[i + 1] - cuts[i], gen_row0=cuts[i])
        sh.bases[i] = cuts[i]
    sh._split = True
    rows_a = _widen(osynth.synth_rows(51, 0, n, 768, "f32"), "f32")
    ix_b, rows_b = _make(rindex, 50_000, 768, "bf16", seed=52)
    q, q32 = _queries(rindex, 12, 768, "f32", seed=53)
    qb, qb32 = _queries(rindex, 12, 768, "bf16", seed=54)
    side = torch.cuda.Stream()
    outs = []
    for rnd, mode in enumerate((1, 2, 1, 2)):
        sh.enable_screen(mode)
        ix_b.enable_screen(mode)
        for i in range(12):
            a = sh.search(q[i:i + 1].contiguous(), 10)
            with torch.cuda.stream(side):
                b = ix_b.search(qb[i:i + 1].contiguous(), 10, stream=side)
            outs.append((rnd, i, a, b))
        assert all(s.search_plan(1, 10) == 11 for s in sh.shards) and ix_b.search_plan(1, 10) == 11
    torch.cuda.synchronize()
    ra64, rb64 = rows_a.astype(np.float64), rows_b.astype(np.float64)
    for rnd, i, a, b in outs:
        for (s, r), rows64, qq in ((a, ra64, q32[i:i + 1]), (b, rb64, qb32[i:i + 1])):
            s, r = s.cpu().numpy(), r.cpu().numpy()
            q64 = qq.astype(np.float64)
            ref_s, ref_r = osearch.topk(q64, rows64, 10)
            probs = osearch.check_topk(s, r, ref_s, ref_r, lambda qi, rr: rows64[rr] @ q64[qi], tol=TOL, tie_band=TIE)
            assert not probs, (rnd, i, probs[:5])
