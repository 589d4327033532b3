"""GPU: the one-launch VALU search (rfx_search on a VALU plan: scan + last-block merge in one
kernel, csrc/k_scan_valu.hip FUSED, per-stream zeroed launch state in rfx_api.hip).

Bars: bit-identical to the three-launch path (rfx_scan_topk + rfx_topk_merge_lists, then the score rule
rfx_rescore_topk) for every
dtype / nq slice shape / k slot / row mask; repeated launches on one stream and launches on a second
stream agree bit-for-bit (the launch state is returned to zero by every launch); config 2's
shape (100k x 768 f32, nq 1, k 10) matches the CPU oracle (check_topk: rows exact outside the
2e-6 tie band, scores within 1e-5)."""
import numpy as np
import pytest
import torch

from oracle import search as osearch
from oracle import synth as osynth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rindex():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import rfx.index as rindex
    return rindex


def three_launch(rindex, ix, q, k, row_mask=None):
    # scan + merge, then the score rule every search answers with (rfx_rescore_topk: fl32 of the f64 dot,
    # score desc, row asc); the one-launch search applies it in its last block
    cs, cr = ix.scan(q, k, row_mask=row_mask)
    return rindex.rescore_topk(ix, q, *rindex.topk_merge(cs, cr, k, list_len=ix.list_len(q.shape[0], k)))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("nq,k", [(1, 1), (1, 10), (3, 16), (8, 10), (37, 64), (256, 10)])
def test_fused_equals_three_launches(rindex, dtype, nq, k):
    if dtype != "f32" and nq > 8:
        pytest.skip("bf16/f16 batches of > 8 queries take the MFMA plans")
    if dtype == "f32" and nq > 16 and k <= 10:
        pytest.skip("f32 batches of > 16 queries (k <= 10) take kernel 9")
    ix = rindex.DeviceIndex(768, dtype)
    ix.add_synthetic(5, 50_003)
    ix.tombstone([0, 17, 50_002])
    q = rindex.synth_rows(6, 0, nq, 768, dtype)
    assert ix.plan(nq, k)[0] == 0
    s3, r3 = three_launch(rindex, ix, q, k)
    for _ in range(3):  # the launch state must come back to zero after every launch
        s1, r1 = ix.search(q, k)
        assert torch.equal(r1, r3) and torch.equal(s1, s3)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        s2, r2 = ix.search(q, k, stream=side)
    side.synchronize()
    assert torch.equal(r2, r3) and torch.equal(s2, s3)
    assert not np.isin(r1.cpu().numpy(), [0, 17, 50_002]).any()


def test_fused_row_mask(rindex):
    ix = rindex.DeviceIndex(768, "f32")
    ix.add_synthetic(9, 20_000)
    words = np.zeros((20_000 + 31) // 32, dtype=np.int32)
    words[10:40] = -1  # rows 320..1279
    m = ix.mask_tensor(words)
    q = rindex.synth_rows(10, 0, 2, 768, "f32")
    s1, r1 = ix.search(q, 10, row_mask=m)
    s3, r3 = three_launch(rindex, ix, q, 10, row_mask=m)
    assert torch.equal(r1, r3) and torch.equal(s1, s3)
    r = r1.cpu().numpy()
    assert ((r >= 320) & (r < 1280)).all()


def test_fused_interleaved_with_other_shapes(rindex):
    """Launch state is per stream and per index: alternating shapes and indices on one stream
    never see each other's bounds or counters."""
    a = rindex.DeviceIndex(768, "f32")
    a.add_synthetic(1, 30_000)
    b = rindex.DeviceIndex(768, "bf16")
    b.add_synthetic(2, 70_000)
    qa = rindex.synth_rows(3, 0, 8, 768, "f32")
    qb = rindex.synth_rows(4, 0, 1, 768, "bf16")
    ref = [three_launch(rindex, a, qa, 10), three_launch(rindex, b, qb, 5), three_launch(rindex, a, qa[:1], 64)]
    for _ in range(4):
        got = [a.search(qa, 10), b.search(qb, 5), a.search(qa[:1], 64)]
        for (gs, gr), (rs, rr) in zip(got, ref):
            assert torch.equal(gr, rr) and torch.equal(gs, rs)


def test_cfg2_shape_against_oracle(rindex):
    n, dim = 100_000, 768
    ix = rindex.DeviceIndex(dim, "f32")
    ix.add_synthetic(42, n)
    q = rindex.synth_rows(43, 0, 1, dim, "f32")
    s, r = ix.search(q, 10)
    rows64 = osynth.to_f64(osynth.synth_rows(42, 0, n, dim, "f32"), "f32")
    q64 = osynth.to_f64(osynth.synth_rows(43, 0, 1, dim, "f32"), "f32")
    ref_s, ref_r = osearch.topk(q64, rows64, 10)
    probs = osearch.check_topk(s.cpu().numpy(), r.cpu().numpy(), ref_s, ref_r,
                               lambda qi, rows: rows64[np.asarray(rows)] @ q64[qi], tol=1e-5, tie_band=2e-6)
    assert not probs, probs[:5]


@pytest.mark.gpu
def test_unaligned_queries_take_the_three_launch_path(rindex):
    """The one-launch kernel reads queries with 16-B loads; a query buffer 4 B off alignment must
    give the same answer (rfx_search routes it through the widening copy)."""
    ix = rindex.DeviceIndex(768, "f32")
    ix.add_synthetic(31, 20_000)
    q = rindex.synth_rows(32, 0, 1, 768, "f32")
    buf = torch.empty(768 + 1, dtype=torch.float32, device=q.device)
    buf[1:].copy_(q[0])
    qu = buf[1:].view(1, 768)
    assert qu.data_ptr() % 16 == 4
    s0, r0 = ix.search(q, 10)
    s1, r1 = ix.search(qu, 10)
    assert torch.equal(r0, r1) and torch.equal(s0, s1)
