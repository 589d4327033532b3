"""GPU parity of the IVF-Flat int8 path (C ABI rfx_ivf_*, csrc/k_ivf.hip) against oracle/ivf.py:
every stage is integer / single-IEEE-op arithmetic, so the bar is BIT-EXACT everywhere —
generated rows, int8 codes and scales, k-means centroids, list assignment, posting lists, and
search scores and rows."""
import numpy as np
import pytest
import torch

from oracle import ivf as oivf
from oracle import search as osearch
from oracle import synth as osynth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rivf():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import rfx.ivf as rivf
    return rivf


def to_np(t, dtype):
    t = t.cpu()
    if dtype == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_synth_clustered_bit_exact(rivf, dtype):
    got = to_np(rivf.synth_clustered(100, 64, 3, 1000, 300, 768, dtype), dtype)
    ref = oivf.clustered_rows(100, 64, 3, 1000, 300, 768, dtype)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("dim", [256, 768, 1000])
def test_quantize_bit_exact(rivf, dtype, dim):
    x = rivf.synth_clustered(5, 16, 9, 0, 257, dim, dtype)
    x[3] = 0  # all-zero row: codes 0, scale 0
    codes, inv = rivf.quantize(x)
    ref_c, ref_inv = oivf.quantize(oivf.stored_to_f32(to_np(x, dtype), dtype))
    assert np.array_equal(codes.cpu().numpy(), ref_c)
    assert np.array_equal(inv.cpu().numpy().view(np.uint32), ref_inv.view(np.uint32))


def build(rivf, n, dim, nlist, iters=4, dtype="bf16", cseed=7, ncenters=48, seed=5, sample_step=2):
    rows = rivf.synth_clustered(cseed, ncenters, seed, 0, n, dim, dtype)
    ix = rivf.IvfIndex(dim, nlist)
    sample = rows[::sample_step].contiguous()
    ix.train(sample, iters=iters)
    ix.add(rows)
    rows_f32 = oivf.stored_to_f32(to_np(rows, dtype), dtype)
    codes, inv = oivf.quantize(rows_f32)
    sc, _ = oivf.quantize(oivf.stored_to_f32(to_np(sample, dtype), dtype))
    qc, fc = oivf.train(sc, nlist, iters)
    return ix, rows, codes, inv, qc, fc


@pytest.mark.parametrize("dim,nlist,iters", [(256, 16, 0), (256, 64, 5), (768, 100, 3), (1024, 130, 2)])
def test_train_assign_lists_bit_exact(rivf, dim, nlist, iters):
    ix, rows, codes, inv, qc, fc = build(rivf, 6000, dim, nlist, iters)
    gqc, gfc = ix.centroids()
    assert np.array_equal(gqc.cpu().numpy(), qc), "k-means centroids differ"
    assert np.array_equal(gfc.cpu().numpy().view(np.uint32), fc.view(np.uint32))
    gc, ginv, glab = ix.codes()
    assert np.array_equal(gc.cpu().numpy(), codes) and np.array_equal(ginv.cpu().numpy(), inv)
    lab = oivf.assign(codes, qc, fc)
    assert np.array_equal(glab.cpu().numpy(), lab)
    off, ids = ix.lists()
    order, ref_off = oivf.build_lists(lab, nlist)
    assert np.array_equal(off.cpu().numpy(), ref_off) and np.array_equal(ids.cpu().numpy(), order)


@pytest.mark.parametrize("dim,nlist", [(256, 32), (768, 64)])
@pytest.mark.parametrize("nq,k,nprobe", [(1, 10, 4), (7, 1, 1), (100, 10, 8), (256, 33, 16), (40, 64, 64)])
def test_search_bit_exact(rivf, dim, nlist, nq, k, nprobe):
    if nprobe > nlist:
        pytest.skip("nprobe > nlist")
    ix, rows, codes, inv, qc, fc = build(rivf, 8000, dim, nlist)
    lab = oivf.assign(codes, qc, fc)
    q = rivf.synth_clustered(7, 48, 77, 0, nq, dim, "bf16")
    qq, qinv = oivf.quantize(oivf.stored_to_f32(to_np(q, "bf16"), "bf16"))
    s, r = ix.search(q, k, nprobe)
    ref_s, ref_r = oivf.search(qq, qinv, codes, inv, lab, qc, fc, nprobe, k)
    assert np.array_equal(r.cpu().numpy(), ref_r)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32))


def test_search_sparse_lists_and_padding(rivf):
    # many lists, few rows: empty lists in the probe set, k above the rows probed -> (-inf, -1)
    ix, rows, codes, inv, qc, fc = build(rivf, 600, 256, 200, iters=2, sample_step=1)
    lab = oivf.assign(codes, qc, fc)
    q = rivf.synth_clustered(7, 48, 78, 0, 33, 256, "f32")
    qq, qinv = oivf.quantize(q.cpu().numpy())
    s, r = ix.search(q, 20, 3)
    ref_s, ref_r = oivf.search(qq, qinv, codes, inv, lab, qc, fc, 3, 20)
    assert np.array_equal(r.cpu().numpy(), ref_r) and np.array_equal(s.cpu().numpy(), ref_s)
    assert (ref_r == -1).any()


def test_incremental_adds_and_set_centroids(rivf):
    # rows added in two batches == one batch; a second index given the first's centroids
    # (the multi-GPU broadcast path) assigns and searches identically
    dim, nlist = 256, 32
    ix, rows, codes, inv, qc, fc = build(rivf, 4000, dim, nlist)
    more = rivf.synth_clustered(7, 48, 6, 0, 1500, dim, "bf16")
    ix.add(more)
    ix2 = rivf.IvfIndex(dim, nlist)
    ix2.set_centroids(ix.centroids()[0])
    ix2.add(torch.cat([rows, more]))
    q = rivf.synth_clustered(7, 48, 79, 0, 50, dim, "bf16")
    s1, r1 = ix.search(q, 10, 6)
    s2, r2 = ix2.search(q, 10, 6)
    assert torch.equal(r1, r2) and torch.equal(s1, s2)
    assert ix.rows == 5500


def test_sharded_ivf_merge_equals_single(rivf):
    # row-sharded IVF with shared centroids: per-shard top-k (global row ids) merged == one index
    from rfx.index import topk_merge
    dim, nlist, n = 256, 32, 6000
    ix, rows, codes, inv, qc, fc = build(rivf, n, dim, nlist)
    q = rivf.synth_clustered(7, 48, 80, 0, 64, dim, "bf16")
    s_full, r_full = ix.search(q, 10, 5)
    parts_s, parts_r = [], []
    for a, b in ((0, 2500), (2500, n)):
        sh = rivf.IvfIndex(dim, nlist)
        sh.set_centroids(ix.centroids()[0])
        sh.add(rows[a:b].contiguous())
        s, r = sh.search(q, 10, 5)
        parts_s.append(s)
        parts_r.append(torch.where(r >= 0, r + a, r))
    ms, mr = topk_merge(torch.cat(parts_s, 1), torch.cat(parts_r, 1), 10)
    assert torch.equal(mr, r_full) and torch.equal(ms, s_full)


def test_recall_vs_bruteforce(rivf):
    # the quality metric of config 5: recall@10 of IVF vs exact brute force on the float rows
    from rfx.index import DeviceIndex
    dim, nlist, n = 768, 64, 30000
    ix, rows, codes, inv, qc, fc = build(rivf, n, dim, nlist, iters=6, ncenters=64, sample_step=4)
    bf = DeviceIndex(dim, "bf16")
    bf.add(rows)
    q = rivf.synth_clustered(7, 64, 81, 0, 200, dim, "bf16")
    _, r_ivf = ix.search(q, 10, 8)
    _, r_bf = bf.search(q, 10)
    r_ivf, r_bf = r_ivf.cpu().numpy(), r_bf.cpu().numpy()
    recall = np.mean([len(set(r_ivf[i]) & set(r_bf[i])) / 10 for i in range(len(r_bf))])
    assert recall >= 0.8, recall


def test_validation(rivf):
    with pytest.raises(ValueError):
        rivf.IvfIndex(300, 16)
    ix = rivf.IvfIndex(256, 16)
    x = rivf.synth_clustered(1, 4, 1, 0, 10, 256, "bf16")
    with pytest.raises(ValueError):
        ix.add(x)  # untrained
    with pytest.raises(ValueError):
        ix.train(x)  # fewer rows than lists
    ix.train(rivf.synth_clustered(1, 4, 1, 0, 64, 256, "bf16"), iters=1)
    ix.add(x)
    with pytest.raises(ValueError):
        ix.search(x, 10, 17)  # nprobe > nlist
    with pytest.raises(ValueError):
        ix.search(x, 65, 4)


@pytest.mark.parametrize("rows_dtype", ["bf16", "f32"])
def test_search_rerank_matches_oracle(rivf, rows_dtype):
    # IVF candidates (bit-exact int8 stage) re-scored against the original rows: same rows as
    # the oracle's f64 re-rank except inside the fp32 tie band, scores within 1e-5
    dim, nlist, k, rk, nprobe = 768, 64, 10, 40, 8
    rows = rivf.synth_clustered(7, 48, 5, 0, 8000, dim, rows_dtype)
    ix = rivf.IvfIndex(dim, nlist)
    ix.train(rows[::2].contiguous(), iters=4)
    ix.add(rows)
    q = rivf.synth_clustered(7, 48, 91, 0, 64, dim, "bf16")
    s, r = ix.search_rerank(q, k, nprobe, rows, rerank_k=rk)
    _, cand = ix.search(q, rk, nprobe)
    rows64 = oivf.stored_to_f32(to_np(rows, rows_dtype), rows_dtype).astype(np.float64)
    q64 = oivf.stored_to_f32(to_np(q, "bf16"), "bf16").astype(np.float64)
    ref_s, ref_r = oivf.rerank(cand.cpu().numpy(), q64, rows64, k)
    probs = osearch.check_topk(s.cpu().numpy(), r.cpu().numpy(), ref_s, ref_r,
                               lambda qi, rr: rows64[rr] @ q64[qi], tol=1e-5, tie_band=2e-6)
    assert not probs, probs[:5]


def test_rerank_lifts_recall(rivf):
    from rfx.index import DeviceIndex
    dim, nlist, n = 768, 64, 30000
    rows = rivf.synth_clustered(7, 64, 5, 0, n, dim, "bf16")
    ix = rivf.IvfIndex(dim, nlist)
    ix.train(rows[::4].contiguous(), iters=6)
    ix.add(rows)
    bf = DeviceIndex(dim, "bf16")
    bf.add(rows)
    q = rivf.synth_clustered(7, 64, 81, 0, 200, dim, "bf16")
    _, r_bf = bf.search(q, 10)
    _, r_ivf = ix.search(q, 10, 8)
    _, r_rr = ix.search_rerank(q, 10, 8, rows)
    r_bf, r_ivf, r_rr = r_bf.cpu().numpy(), r_ivf.cpu().numpy(), r_rr.cpu().numpy()
    rec = lambda r: np.mean([len(set(r[i]) & set(r_bf[i])) / 10 for i in range(len(r_bf))])
    assert rec(r_rr) >= rec(r_ivf) and rec(r_rr) >= 0.97, (rec(r_ivf), rec(r_rr))


def test_save_load_roundtrip(rivf, tmp_path):
    ix, rows, codes, inv, qc, fc = build(rivf, 5000, 256, 32)
    q = rivf.synth_clustered(7, 48, 92, 0, 40, 256, "bf16")
    s1, r1 = ix.search(q, 10, 6)
    path = str(tmp_path / "ivf.rfx")
    ix.save(path)
    ix2 = rivf.IvfIndex.load(path)
    assert ix2.rows == ix.rows and ix2.trained and ix2.nlist == 32
    s2, r2 = ix2.search(q, 10, 6)
    assert torch.equal(r1, r2) and torch.equal(s1, s2)
    assert torch.equal(ix2.centroids()[1], ix.centroids()[1])
    with pytest.raises(RuntimeError):
        (tmp_path / "bad.rfx").write_bytes(b"RFXIDX01garbage")
        rivf.IvfIndex.load(str(tmp_path / "bad.rfx"))
