"""GPU: the exact two-pass scan (kernel 10 + k_screen.hip) through the C ABI.

Bars: the int8 copy is BIT-EXACT with oracle/screen.py (codes, tile scales, live words; the two
norm maxima to f64 rounding); searches return the brute-force top-k of oracle/search.py under the
same parity rule as every scan (check_topk: rows identical outside the 2e-6 tie band, no
duplicates, scores within 1e-5 of the f64 score); the exact scan (screen off) and the forced
fallback return the same rows."""
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


def _make(rindex, n, d, dtype, seed=21, screen=1):
    ix = rindex.DeviceIndex(d, dtype)
    ix.add_synthetic(seed, n)
    if screen:
        ix.enable_screen(screen)
    rows32 = _widen(osynth.synth_rows(seed, 0, n, d, dtype), dtype)
    return ix, rows32


def _queries(rindex, nq, d, dtype, seed=22):
    return rindex.synth_rows(seed, 0, nq, d, dtype), _widen(osynth.synth_rows(seed, 0, nq, d, dtype), dtype)


@pytest.mark.parametrize("dtype,d", [("bf16", 768), ("f16", 768), ("bf16", 1024), ("f16", 1024)])
def test_int8_copy_bit_exact(rindex, dtype, d):
    n = 5000 + 17  # ragged last tile
    ix, rows32 = _make(rindex, n, d, dtype)
    ix.tombstone([3, 64, 5000])
    rows32[[3, 64, 5000]] = np.nan
    nt = (n + 31) // 32
    codes, scales, live, stats = ix.screen_read(0, nt)
    rc, rs, rl, rst = oscreen.quantize_tiles(rows32)
    assert codes.tobytes() == rc.tobytes()
    assert scales.tobytes() == rs.tobytes()
    assert live.tobytes() == rl.tobytes()
    assert np.allclose(stats[:2], rst[:2], rtol=2e-7, atol=0) and stats[2] == rst[2] == scales.max()


@pytest.mark.parametrize("nq,k", [(256, 10), (100, 10), (300, 4), (256, 1)])
def test_two_pass_matches_oracle_768(rindex, nq, k):
    ix, rows32 = _make(rindex, 40000, 768, "bf16")
    assert ix.search_plan(nq, k) == 10
    q, q32 = _queries(rindex, nq, 768, "bf16")
    _check(ix, rows32, q, q32, k)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_two_pass_matches_oracle_1024(rindex, dtype):
    ix, rows32 = _make(rindex, 30000, 1024, dtype)
    assert ix.search_plan(256, 10) == 10
    q, q32 = _queries(rindex, 256, 1024, dtype)
    _check(ix, rows32, q, q32, 10)


def test_two_pass_equals_exact_scan_and_forced_fallback(rindex):
    ix, rows32 = _make(rindex, 50000, 768, "bf16")
    q, q32 = _queries(rindex, 256, 768, "bf16")
    s1, r1 = _check(ix, rows32, q, q32, 10)
    ws = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
    ix.search(q, 10, workspace=ws)
    diag, fb = ix.screen_diag(256, 10, ws)
    assert not fb and (diag[:, 1] >= 10).all() and (diag[:, 1] < 2000).all()
    ix.enable_screen(2)  # every batch through the gated exact pass
    s2, r2 = _check(ix, rows32, q, q32, 10)
    ix.search(q, 10, workspace=ws)
    assert ix.screen_diag(256, 10, ws)[1]
    ix.enable_screen(0)
    assert ix.search_plan(256, 10) == 6
    s3, r3 = _check(ix, rows32, q, q32, 10)
    assert np.array_equal(r1, r3) and np.array_equal(r2, r3)


def test_appends_tombstones_and_ties(rindex):
    ix, rows32 = _make(rindex, 3000, 768, "bf16")
    q, q32 = _queries(rindex, 200, 768, "bf16")
    # appended rows land in the half-filled last tile (its scale is recomputed) and beyond
    ix.add_synthetic(21, 2500)
    rows32 = _widen(osynth.synth_rows(21, 0, 5500, 768, "bf16"), "bf16")
    # exact duplicates of query 0's winner (tie rule: lower row first), then tombstone some rows
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    dup = ix.read(top, 1)
    first = ix.add(dup.repeat(3, 1))
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 3, axis=0)])
    dead = [top + 1, 4000, first + 1]
    ix.tombstone(dead)
    rows32[dead] = np.nan
    s, r = _check(ix, rows32, q, q32, 10)
    assert r[0, 0] == top and r[0, 1] == first and r[0, 2] == first + 2
    codes, scales, live, _ = ix.screen_read(0, (rows32.shape[0] + 31) // 32)
    rc, rs, rl, _ = oscreen.quantize_tiles(rows32)
    assert codes.tobytes() == rc.tobytes() and scales.tobytes() == rs.tobytes() and live.tobytes() == rl.tobytes()


def test_duplicate_heavy_corpus_takes_the_fallback_correctly(rindex):
    """40 copies of one row inside one workgroup's lists overflow the lane lists: the select kernel
    must send the batch to the exact pass, and the result must still be exact."""
    ix, rows32 = _make(rindex, 20000, 768, "bf16", screen=0)
    q, q32 = _queries(rindex, 256, 768, "bf16")
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    first = ix.add(ix.read(top, 1).repeat(40, 1))
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 40, axis=0)])
    ix.enable_screen(1)
    s, r = _check(ix, rows32, q, q32, 10)
    assert r[0, 0] == top and list(r[0, 1:]) == list(range(first, first + 9))


def test_row_mask_with_two_pass(rindex):
    ix, rows32 = _make(rindex, 12000, 768, "bf16")
    q, q32 = _queries(rindex, 256, 768, "bf16")
    rng = np.random.default_rng(3)
    allowed = rng.random(12000) < 0.3
    words = np.zeros((12000 + 31) // 32, dtype=np.uint32)
    for i in np.nonzero(allowed)[0]:
        words[i >> 5] |= np.uint32(1 << (i & 31))
    m = torch.from_numpy(words.view(np.int32)).cuda()
    _check(ix, rows32, q, q32, 10, row_mask=m, allowed=allowed)


def test_search_records_row_offset(rindex):
    ix, rows32 = _make(rindex, 8000, 768, "bf16")
    q, q32 = _queries(rindex, 256, 768, "bf16")
    s, r = ix.search(q, 10)
    rec = ix.search_records(q, 10, row_offset=1_000_000)
    torch.cuda.synchronize()
    rec = rec.cpu().numpy()
    assert np.array_equal(rec[..., 1], r.cpu().numpy() + 1_000_000)
    assert np.array_equal((rec[..., 0] & 0xffffffff).astype(np.uint32).view(np.float32), s.cpu().numpy())


@pytest.mark.parametrize("mode", [1, 2])
def test_scores_rows_form_with_row_offset_equals_records(rindex, mode):
    """rfx_search_timed writing (scores, rows) with a row offset — through the select, and through the
    forced gated fallback (mode 2), whose merge adds the offset and whose re-score must subtract it
    again before it reads the shard's rows — equals the records form."""
    from rfx._lib import check, lib, ptr, stream_ptr

    ix, _ = _make(rindex, 9000, 768, "bf16", screen=mode)
    q, _ = _queries(rindex, 256, 768, "bf16")
    off = 1000
    rec = ix.search_records(q, 10, row_offset=off)
    ws = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
    s = torch.empty((256, 10), dtype=torch.float32, device="cuda")
    r = torch.empty((256, 10), dtype=torch.int64, device="cuda")
    check(lib.rfx_search_timed(ix.handle, ptr(q), 256, 10, None, 0, off, ptr(s), ptr(r), None, ptr(ws), ws.numel(),
                               stream_ptr(None), None, None))
    torch.cuda.synchronize()
    assert ix.screen_diag(256, 10, ws)[1] == (mode == 2)
    rec = rec.cpu().numpy()
    assert np.array_equal(rec[..., 1], r.cpu().numpy())
    assert np.array_equal((rec[..., 0] & 0xffffffff).astype(np.uint32).view(np.float32), s.cpu().numpy())
    ix.enable_screen(1)


def test_small_and_empty(rindex):
    ix = rindex.DeviceIndex(768, "bf16")
    ix.enable_screen(1)
    q, q32 = _queries(rindex, 256, 768, "bf16")
    s, r = ix.search(q, 10)  # no rows: the exact padding path
    assert (r.cpu().numpy() == -1).all()
    ix.add_synthetic(21, 7)  # fewer live rows than k
    rows32 = _widen(osynth.synth_rows(21, 0, 7, 768, "bf16"), "bf16")
    s, r = _check(ix, rows32, q, q32, 10)
    assert (r[:, 7:] == -1).all()


def test_staged_search_on_two_streams_equals_one_call():
    """rfx_search_staged: stage 1 (quantiser + kernel 10, on fewer workgroups) on one stream, stage 2
    (select + gated fallback) on another, ordered by an event, writes the same records as one
    rfx_search_records call — including a forced fallback, and a VALU plan (stage 1 = the whole search)."""
    import ctypes

    from rfx._lib import check, lib, ptr
    from rfx.index import DeviceIndex, synth_rows

    ix = DeviceIndex(768, "bf16", 0)
    ix.add_synthetic(31, 150_000)
    ix.enable_screen(1)
    for nq, mode in ((256, 1), (256, 2), (3, 1)):
        ix.enable_screen(mode)
        q = synth_rows(32, 0, nq, 768, "bf16")
        ref = ix.search_records(q, 10, row_offset=1000)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for blocks in (0, 248, 77):
            ws = torch.empty(ix.workspace_bytes(nq, 10), dtype=torch.uint8, device="cuda")
            out = torch.full((nq, 10, 2), 7, dtype=torch.int64, device="cuda")
            ev = torch.cuda.Event()
            s1.wait_stream(torch.cuda.current_stream())
            check(lib.rfx_search_staged(ix.handle, ptr(q), nq, 10, None, 0, 1000, None, None, ptr(out), ptr(ws),
                                        ws.numel(), 1, blocks, ctypes.c_void_p(s1.cuda_stream)))
            ev.record(s1)
            s2.wait_event(ev)
            check(lib.rfx_search_staged(ix.handle, ptr(q), nq, 10, None, 0, 1000, None, None, ptr(out), ptr(ws),
                                        ws.numel(), 2, blocks, ctypes.c_void_p(s2.cuda_stream)))
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (nq, mode, blocks)
    ix.enable_screen(1)


def test_xcd_balanced_split_is_exact_across_launches_and_streams(rindex):
    """Kernel 10's XCD-balanced tile split (>= 64 tiles per block: 600k rows) moves tiles between XCDs
    from launch to launch as the measured speeds change the weights; every launch's answer must be
    the same (bit for bit) and hold the exact scan's rows, also with two streams searching at once
    (each launch reads its own weight snapshot)."""
    n = 600_000
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(31, n)
    q1 = rindex.synth_rows(32, 0, 256, 768, "bf16")
    q2 = rindex.synth_rows(33, 0, 256, 768, "bf16")
    ix.enable_screen(0)
    ex1, ex2 = ix.search(q1, 10), ix.search(q2, 10)
    ix.enable_screen(1)
    assert ix.search_plan(256, 10) == 10
    ref1 = ix.search(q1, 10)

    def same_rows(a, b):  # the exact scan's f32 sums may order an f32 tie differently: compare as sets
        return torch.equal(torch.sort(a, dim=1)[0], torch.sort(b, dim=1)[0])

    assert same_rows(ref1[1], ex1[1])
    for _ in range(6):  # the weights move between these launches
        s, r = ix.search(q1, 10)
        assert torch.equal(s, ref1[0]) and torch.equal(r, ref1[1])
    ref2 = ix.search(q2, 10)
    assert same_rows(ref2[1], ex2[1])
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    wa = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
    wb = torch.empty_like(wa)
    torch.cuda.synchronize()
    outs = []
    for _ in range(4):
        outs.append((ix.search(q1, 10, workspace=wa, stream=sa), ix.search(q2, 10, workspace=wb, stream=sb)))
    torch.cuda.synchronize()
    for (s1, r1), (s2, r2) in outs:
        assert torch.equal(s1, ref1[0]) and torch.equal(r1, ref1[1])
        assert torch.equal(s2, ref2[0]) and torch.equal(r2, ref2[1])
