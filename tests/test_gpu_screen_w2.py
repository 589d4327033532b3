"""GPU: the two-pass scan for the micro-batcher's batch sizes: batches of 9..64 questions
(rfx/batcher.py forms them from <= 50 concurrent chat threads per process, config.py:137, chat.py:496-521)
run the 2-wave kernel 10 (64 queries per workgroup, two workgroups per CU, k_scan_screen.h NW = 2) and the
select; the gated fallback is the exact kernel 6 (bf16 / f16, d 768), 8 (d 1024) or 9 (f32) padded to its
query groups.  f32 stores take the two-pass scan too (the quantiser and the select read f32 queries and
rows; the re-score multiplies them in f64).

Bars as tests/test_gpu_screen.py: the brute-force top-k of oracle/search.py under check_topk (rows identical
outside the 2e-6 tie band, scores within 1e-5 of the f64 score), the forced fallback and the exact scan
return the same rows, and the 2-wave answer equals the 8-wave one bit for bit where both apply."""
import numpy as np
import pytest
import torch

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


def _make(rindex, n, d, dtype, seed=21, screen=1):
    ix = rindex.DeviceIndex(d, dtype)
    ix.add_synthetic(seed, n)
    if screen:
        ix.enable_screen(screen)
    return ix, _widen(osynth.synth_rows(seed, 0, n, d, dtype), dtype)


def _queries(rindex, nq, d, dtype, seed=22):
    return rindex.synth_rows(seed, 0, nq, d, dtype), _widen(osynth.synth_rows(seed, 0, nq, d, dtype), dtype)


def _check(ix, rows32, q, q32, k, row_mask=None, allowed=None, workspace=None):
    s, r = ix.search(q, k, row_mask=row_mask, workspace=workspace)
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


@pytest.mark.parametrize("dtype,d,n,nq,k", [
    ("bf16", 768, 60_000, 9, 10), ("bf16", 768, 60_000, 16, 10), ("bf16", 768, 60_000, 32, 4),
    ("bf16", 768, 60_000, 64, 10), ("bf16", 768, 60_000, 40, 1), ("f16", 768, 30_000, 33, 10),
    ("bf16", 1024, 30_000, 48, 10), ("f16", 1024, 30_000, 17, 4),
    ("f32", 768, 100_000, 16, 10), ("f32", 768, 100_000, 32, 10), ("f32", 768, 100_000, 64, 10),
    ("f32", 768, 20_000, 9, 10), ("f32", 1024, 20_000, 24, 10)])
def test_w2_matches_oracle(rindex, dtype, d, n, nq, k):
    ix, rows32 = _make(rindex, n, d, dtype)
    plan = ix.search_plan(nq, k)
    if dtype == "f32" and d == 1024:
        assert plan != 10  # (no exact batched f32 kernel at d 1024 for the fallback: the exact plan)
    else:
        assert plan == 10, plan
    q, q32 = _queries(rindex, nq, d, dtype)
    ws = torch.empty(ix.workspace_bytes(nq, k), dtype=torch.uint8, device="cuda")
    _check(ix, rows32, q, q32, k, workspace=ws)
    if plan == 10:
        diag, fb = ix.screen_diag(nq, k, ws)
        assert not fb and (diag[:, 1] >= min(k, n)).all(), (fb, diag[:, 1].min())
    ix.close()


@pytest.mark.parametrize("dtype,d", [("bf16", 768), ("bf16", 1024), ("f32", 768)])
def test_w2_forced_fallback_and_exact_scan(rindex, dtype, d):
    """The gated fallback of each store type (kernel 6 / 8 / 9, padded to 256 / 128 / 128 queries, its
    threshold table zeroed by the quantiser over that padded batch) and the exact scan: the same rows."""
    nq = 32
    ix, rows32 = _make(rindex, 40_000, d, dtype)
    q, q32 = _queries(rindex, nq, d, dtype)
    s1, r1 = _check(ix, rows32, q, q32, 10)
    ix.enable_screen(2)  # every batch through the gated exact pass
    ws = torch.empty(ix.workspace_bytes(nq, 10), dtype=torch.uint8, device="cuda")
    s2, r2 = _check(ix, rows32, q, q32, 10, workspace=ws)
    assert ix.screen_diag(nq, 10, ws)[1]
    ix.enable_screen(0)
    assert ix.search_plan(nq, 10) != 10
    s3, r3 = _check(ix, rows32, q, q32, 10)
    assert np.array_equal(r1, r3) and np.array_equal(r2, r3)
    # one score rule: the two-pass answer, the fallback's and the exact scan's scores are the same bits
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32)) and np.array_equal(s1.view(np.uint32), s3.view(np.uint32))
    ix.close()


def test_w2_duplicate_heavy_corpus_takes_the_fallback(rindex):
    ix, rows32 = _make(rindex, 20_000, 768, "bf16", screen=0)
    q, q32 = _queries(rindex, 24, 768, "bf16")
    top = int(osearch.topk(q32[:1].astype(np.float64), rows32.astype(np.float64), 1)[1][0, 0])
    first = ix.add(ix.read(top, 1).repeat(40, 1))
    rows32 = np.concatenate([rows32, np.repeat(rows32[top:top + 1], 40, axis=0)])
    ix.enable_screen(1)
    s, r = _check(ix, rows32, q, q32, 10)
    assert r[0, 0] == top and list(r[0, 1:]) == list(range(first, first + 9))
    ix.close()


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_w2_row_mask_appends_tombstones(rindex, dtype):
    ix, rows32 = _make(rindex, 12_000, 768, dtype)
    ix.add_synthetic(21, 3_000)  # appended rows: the last tile re-quantised
    rows32 = _widen(osynth.synth_rows(21, 0, 15_000, 768, dtype), dtype)
    dead = [5, 777, 14_999]
    ix.tombstone(dead)
    rows32[dead] = np.nan
    q, q32 = _queries(rindex, 50, 768, dtype)
    rng = np.random.default_rng(3)
    allowed = rng.random(15_000) < 0.3
    words = np.zeros((15_000 + 31) // 32, dtype=np.uint32)
    for i in np.nonzero(allowed)[0]:
        words[i >> 5] |= np.uint32(1 << (i & 31))
    m = torch.from_numpy(words.view(np.int32)).cuda()
    _check(ix, rows32, q, q32, 10, row_mask=m, allowed=allowed)
    _check(ix, rows32, q, q32, 10)
    ix.close()


def test_w2_records_row_offset_and_eight_wave_equality(rindex):
    """search_records of a 2-wave batch carries the row offset; a 2-wave batch's answer equals the same
    queries' rows of an 8-wave batch (nq 256), bit for bit, on a store large enough for the XCD-balanced
    split of both kernels (>= 64 tiles per workgroup: 1.1M rows)."""
    n = 1_100_000
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(31, n)
    ix.enable_screen(1)
    q = rindex.synth_rows(32, 0, 256, 768, "bf16")
    s8, r8 = ix.search(q, 10)
    for nq in (9, 32, 64):
        for _ in range(3):  # the XCD weights move between launches: every split is exact
            s, r = ix.search(q[:nq].contiguous(), 10)
            assert torch.equal(s, s8[:nq]) and torch.equal(r, r8[:nq]), nq
    rec = ix.search_records(q[:32].contiguous(), 10, row_offset=1_000_000)
    torch.cuda.synchronize()
    rec = rec.cpu().numpy()
    assert np.array_equal(rec[..., 1], r8[:32].cpu().numpy() + 1_000_000)
    assert np.array_equal((rec[..., 0] & 0xffffffff).astype(np.uint32).view(np.float32), s8[:32].cpu().numpy())
    ix.enable_screen(0)
    se, re_ = ix.search(q[:32].contiguous(), 10)
    assert torch.equal(torch.sort(re_, dim=1)[0], torch.sort(r8[:32], dim=1)[0])
    ix.close()
