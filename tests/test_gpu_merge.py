"""GPU: the top-k merge kernels through the C ABI — list-structured merge (heads prefilter),
packed all-gather records and the gathered merge of the multi-GPU step — against a numpy
oracle merge (score desc, row asc; the tie rule of oracle/search.py)."""
import numpy as np
import pytest
import torch

from rfx import dist as rdist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rindex():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import rfx.index as ri
    return ri


def oracle_merge(s, r, k):
    """numpy reference: drop sentinel rows (< 0 or int32 max), sort by (-score, row)."""
    nq = s.shape[0]
    out_s = np.full((nq, k), -np.inf, dtype=np.float32)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    for i in range(nq):
        live = (r[i] >= 0) & (r[i] != 0x7fffffff) & (r[i] != 0x7fffffffffffffff)
        order = np.lexsort((r[i][live], -s[i][live].astype(np.float64)))[:k]
        out_s[i, :len(order)] = s[i][live][order]
        out_r[i, :len(order)] = r[i][live][order]
    return out_s, out_r


def sorted_lists(rng, nq, n_lists, L, rows_total, empty_frac=0.1, ties=False):
    """n_lists sorted lists of length L per query (best first), distinct rows, some empty tails."""
    s = rng.standard_normal((nq, n_lists, L)).astype(np.float32)
    if ties:
        s = np.round(s * 8) / 8  # many equal scores: the row tie-break decides
    s = -np.sort(-s, axis=2)
    r = np.stack([rng.permutation(rows_total)[: n_lists * L] for _ in range(nq)]).reshape(nq, n_lists, L)
    r = r.astype(np.int64)
    if ties:  # within equal scores a list is ordered by row asc, as the scan writes it
        for q in range(nq):
            for j in range(n_lists):
                o = np.lexsort((r[q, j], -s[q, j].astype(np.float64)))
                s[q, j], r[q, j] = s[q, j][o], r[q, j][o]
    cut = rng.random((nq, n_lists)) < empty_frac
    for q, j in zip(*np.nonzero(cut)):
        m = rng.integers(0, L)
        s[q, j, m:] = -np.inf
        r[q, j, m:] = 0x7fffffff
    return s.reshape(nq, -1), r.reshape(nq, -1)


@pytest.mark.parametrize("L,k", [(10, 10), (10, 5), (4, 4), (4, 1), (16, 16), (16, 12)])
@pytest.mark.parametrize("ties", [False, True])
def test_merge_lists_matches_oracle(rindex, L, k, ties):
    rng = np.random.default_rng(L * 100 + k + ties)
    s, r = sorted_lists(rng, 37, 512, L, 10_000_000, ties=ties)
    ref_s, ref_r = oracle_merge(s, r, k)
    cs = torch.from_numpy(s).cuda()
    for rows_dtype in (torch.int32, torch.int64):
        cr = torch.from_numpy(r).to(rows_dtype).cuda()
        for ll, srt in ((L, False), (1, False), (L, True)):
            out_s, out_r = rindex.topk_merge(cs, cr, k, list_len=ll, sorted=srt)
            assert np.array_equal(out_r.cpu().numpy(), ref_r), (ll, rows_dtype, srt)
            assert np.array_equal(out_s.cpu().numpy(), ref_s)


def test_merge_lists_hint_on_unsorted_input_stays_exact(rindex):
    """list_len is only a hint: on lists that are NOT sorted the result is still exact."""
    rng = np.random.default_rng(3)
    s = rng.standard_normal((16, 5120)).astype(np.float32)
    r = np.stack([rng.permutation(1 << 20)[:5120] for _ in range(16)]).astype(np.int64)
    ref_s, ref_r = oracle_merge(s, r, 10)
    out_s, out_r = rindex.topk_merge(torch.from_numpy(s).cuda(), torch.from_numpy(r).cuda(), 10, list_len=10)
    assert np.array_equal(out_r.cpu().numpy(), ref_r)


def test_merge_row_offset_and_empty_queries(rindex):
    s = np.full((3, 40), -np.inf, dtype=np.float32)
    r = np.full((3, 40), 0x7fffffff, dtype=np.int64)
    s[1, :4] = [0.5, 0.25, 0.125, 0.0]
    r[1, :4] = [7, 3, 9, 1]
    out_s, out_r = rindex.topk_merge(torch.from_numpy(s).cuda(), torch.from_numpy(r).to(torch.int32).cuda(), 5,
                                     row_offset=1000, list_len=10)
    out_r = out_r.cpu().numpy()
    assert (out_r[0] == -1).all() and (out_r[2] == -1).all()
    assert out_r[1].tolist() == [1007, 1003, 1009, 1001, -1]


def test_merge_records_layout_is_dist_pack(rindex):
    rng = np.random.default_rng(5)
    s, r = sorted_lists(rng, 9, 64, 10, 1 << 20)
    cs, cr = torch.from_numpy(s).cuda(), torch.from_numpy(r).to(torch.int32).cuda()
    out_s, out_r = rindex.topk_merge(cs, cr, 10, row_offset=123, list_len=10)
    rec = rindex.topk_merge_records(cs, cr, 10, row_offset=123, list_len=10)
    ref = rdist.pack(out_s, out_r)
    assert torch.equal(rec[..., 1], ref[..., 1])
    assert torch.equal(rec[..., 0].to(torch.int32), ref[..., 0].to(torch.int32))  # score bits (low word)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_merge_gathered_equals_flat_merge(rindex, world):
    """The multi-GPU exchange on one device: shards' records stacked as the all-gather lays them
    out, merged by rfx_merge_gathered, equal the merge of every shard's candidates at once."""
    rng = np.random.default_rng(world)
    nq, k = 21, 10
    shards = [sorted_lists(rng, nq, 32, 10, 1 << 20) for _ in range(world)]
    recs = []
    for w, (s, r) in enumerate(shards):
        cs, cr = torch.from_numpy(s).cuda(), torch.from_numpy(r).to(torch.int32).cuda()
        recs.append(rindex.topk_merge_records(cs, cr, k, row_offset=w * (1 << 20), list_len=10))
    out_s, out_r = rindex.merge_gathered(torch.stack(recs), k)
    all_s = np.concatenate([s for s, _ in shards], axis=1)
    all_r = np.concatenate([np.where(r == 0x7fffffff, r, r + w * (1 << 20)) for w, (_, r) in enumerate(shards)], axis=1)
    ref_s, ref_r = oracle_merge(all_s, all_r, k)
    assert np.array_equal(out_r.cpu().numpy(), ref_r)
    assert np.array_equal(out_s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("world,k,ties", [(1, 1, False), (2, 5, True), (8, 10, False), (8, 10, True), (5, 16, True),
                                          (8, 64, False), (16, 32, True), (9, 64, False), (64, 10, True)])
def test_merge_gathered_shapes_and_ties(rindex, world, k, ties):
    """rfx_merge_gathered on sorted per-rank records (the dedicated one-wave-per-query kernel up to
    world * k = 512, the block merge beyond): ties across ranks, short lists padded (-inf, -1), nq not
    a multiple of the kernel's 4 queries per block."""
    rng = np.random.default_rng(world * 1000 + k + ties)
    nq = 23
    recs, all_s, all_r = [], [], []
    for w in range(world):
        s, r = sorted_lists(rng, nq, 1, k, 1 << 20, empty_frac=0.3, ties=ties)
        r = np.where(r == 0x7fffffff, -1, r + w * (1 << 20))
        s = np.where(r < 0, -np.inf, s).astype(np.float32)
        recs.append(rdist.pack(torch.from_numpy(s).cuda(), torch.from_numpy(r).cuda()))
        all_s.append(s)
        all_r.append(r)
    out_s, out_r = rindex.merge_gathered(torch.stack(recs), k)
    ref_s, ref_r = oracle_merge(np.concatenate(all_s, axis=1), np.concatenate(all_r, axis=1), k)
    assert np.array_equal(out_r.cpu().numpy(), ref_r)
    assert np.array_equal(out_s.cpu().numpy(), ref_s)


def test_scan_then_records_then_gathered_equals_search(rindex):
    """Sharded search on one device (2 shards of one corpus) == unsharded search."""
    n, d = 40_000, 768
    full = rindex.DeviceIndex(d, "bf16")
    full.add_synthetic(11, n)
    q = rindex.synth_rows(12, 0, 256, d, "bf16")
    ref_s, ref_r = full.search(q, 10)
    recs = []
    for r0, r1 in (rdist.shard_range(n, 0, 2), rdist.shard_range(n, 1, 2)):
        ix = rindex.DeviceIndex(d, "bf16")
        ix.add_synthetic(11, r1 - r0, gen_row0=r0)
        cs, cr = ix.scan(q, 10)
        rec = rindex.topk_merge_records(cs, cr, 10, row_offset=r0, list_len=ix.list_len(256, 10))
        recs.append(rindex.rescore_topk(ix, q, records=rec, row_offset=r0))  # the search's score rule
    s, r = rindex.merge_gathered(torch.stack(recs), 10)
    assert torch.equal(r, ref_r)
    assert torch.equal(s, ref_s)


@pytest.mark.parametrize("nq,n_lists,L,k", [(1, 391, 16, 10), (1, 3000, 16, 16), (3, 391, 16, 5), (32, 700, 10, 10),
                                            (7, 130, 16, 10), (1, 129, 16, 10), (2, 5000, 4, 4), (33, 512, 10, 10)])
@pytest.mark.parametrize("ties", [False, True])
def test_merge_few_queries_many_lists_matches_oracle(rindex, nq, n_lists, L, k, ties):
    """Few queries over many candidate lists (config 2's shape: 1 query, 391 lists of 16), where
    the heads bound does most of the pruning; equal to the oracle for every list_len hint,
    with empty list tails and tied scores."""
    rng = np.random.default_rng(nq * 7919 + n_lists * 31 + L + k + ties)
    s, r = sorted_lists(rng, nq, n_lists, L, 10_000_000, empty_frac=0.2, ties=ties)
    ref_s, ref_r = oracle_merge(s, r, k)
    for rows_dtype in (torch.int32, torch.int64):
        for ll, srt in ((L, False), (1, False), (L, True)):
            cs = torch.from_numpy(s.copy()).cuda()
            cr = torch.from_numpy(r).to(rows_dtype).cuda()
            out_s, out_r = rindex.topk_merge(cs, cr, k, list_len=ll, row_offset=5, sorted=srt)
            assert np.array_equal(out_r.cpu().numpy(), np.where(ref_r >= 0, ref_r + 5, -1)), (ll, rows_dtype, srt)
            assert np.array_equal(out_s.cpu().numpy(), ref_s)
            if srt:  # the records form of the sorted merge carries the same rows and scores
                rec = rindex.topk_merge_records(cs, cr, k, list_len=ll, row_offset=5, sorted=True)
                rs, rr = rdist.unpack(rec.unsqueeze(0))
                assert torch.equal(rr, out_r) and torch.equal(rs, out_s)


def test_merge_heads_bound_unsorted_and_all_empty(rindex):
    rng = np.random.default_rng(11)
    s = rng.standard_normal((2, 6400)).astype(np.float32)
    r = np.stack([rng.permutation(10**6)[:6400] for _ in range(2)]).astype(np.int64)
    s[1] = -np.inf  # query 1: nothing live
    r[1] = 0x7fffffff
    ref_s, ref_r = oracle_merge(s, r, 10)
    cs, cr = torch.from_numpy(s.copy()).cuda(), torch.from_numpy(r).to(torch.int32).cuda()
    out_s, out_r = rindex.topk_merge(cs, cr, 10, list_len=16)  # wrong hint: unsorted lists
    assert np.array_equal(out_r.cpu().numpy(), ref_r) and np.array_equal(out_s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("dtype,nq", [("f32", 1), ("f32", 8), ("bf16", 1), ("bf16", 32), ("bf16", 100),
                                      ("bf16", 256), ("f16", 200)])
def test_sorted_merge_of_every_scan_plan(rindex, dtype, nq):
    """Every scan kernel writes sorted lists: the sorted merge of its candidates equals the exact
    (unsorted-safe) merge bit for bit, with tombstones and a row mask in play."""
    ix = rindex.DeviceIndex(768, dtype)
    ix.add_synthetic(21, 40_001)
    ix.tombstone(list(range(0, 40_001, 97)))
    q = rindex.synth_rows(22, 0, nq, 768, dtype)
    words = np.full((40_001 + 31) // 32, -1, dtype=np.int32)
    words[5:40] = 0
    for m in (None, ix.mask_tensor(words)):
        for k in (1, 10):
            cs, cr = ix.scan(q, k, row_mask=m)
            ll = ix.list_len(nq, k)
            a_s, a_r = rindex.topk_merge(cs, cr, k, list_len=ll)
            b_s, b_r = rindex.topk_merge(cs, cr, k, list_len=ll, sorted=True)
            assert torch.equal(a_r, b_r) and torch.equal(a_s, b_s), (ix.plan(nq, k), m is None, k)
            # the search applies the one score rule (fl32 of the f64 dot, score desc / row asc) to its final
            # k; the merged scan candidates carry the scan's f32 sums until rescore_topk applies it
            c_s, c_r = ix.search(q, k, row_mask=m)
            e_s, e_r = rindex.rescore_topk(ix, q, a_s.clone(), a_r.clone())
            assert torch.equal(c_r, e_r) and torch.equal(c_s, e_s), (ix.plan(nq, k), m is None, k)
