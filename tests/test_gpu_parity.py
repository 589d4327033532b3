"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same seeded inputs.

Bars: generated rows, projection weights and embeddings are BIT-EXACT;
search returns identical row lists except inside the documented tie band (|Δscore| <= 2e-6,
oracle check_topk) and scores within 1e-5 of the oracle's fp64 score of the same row.
"""
import numpy as np
import pytest
import torch

from oracle import embed as oembed
from oracle import search as osearch
from oracle import synth as osynth
from oracle import textproc

pytestmark = pytest.mark.gpu

TOL = 1e-5      # |gpu score - fp64 oracle score|, north_star's fp32 tolerance
TIE = 2e-6      # tie band for index order (fp32 accumulation-order noise at d <= 1024)


@pytest.fixture(scope="module")
def rfx():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import rfx.index as rindex
    import rfx.embedder as remb
    return rindex, remb


def stored_to_np(t: torch.Tensor, dtype: str) -> np.ndarray:
    t = t.cpu()
    if dtype == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def run_search_check(rindex, n, dim, dtype, nq, k, seed=7, qseed=8, dup=None, tomb=None, row_block=1 << 16):
    ix = rindex.DeviceIndex(dim, dtype)
    if n:
        ix.add_synthetic(seed, n)
    rows_np = osynth.synth_rows(seed, 0, n, dim, dtype)
    if dup:
        # plant exact duplicate rows to pin the tie rule (lower row id first)
        src, dst = dup
        vec = ix.read(src, 1)
        ix2 = rindex.DeviceIndex(dim, dtype)
        all_rows = ix.read(0, n)
        all_rows[dst] = vec[0]
        ix2.add(all_rows)
        ix = ix2
        rows_np = rows_np.copy()
        rows_np[dst] = rows_np[src]
    rows64 = osynth.to_f64(rows_np, dtype)
    if tomb is not None and len(tomb):
        ix.tombstone(tomb)
        rows64 = rows64.copy()
        rows64[np.asarray(tomb)] = np.nan
    q = rindex.synth_rows(qseed, 0, nq, dim, dtype)
    q64 = osynth.to_f64(osynth.synth_rows(qseed, 0, nq, dim, dtype), dtype)
    s, r = ix.search(q, k)
    torch.cuda.synchronize()
    s, r = s.cpu().numpy(), r.cpu().numpy()
    ref_s, ref_r = osearch.topk(q64, rows64, k, row_block=row_block)

    def scores_of(qi, rows):
        return rows64[rows] @ q64[qi]

    probs = osearch.check_topk(s, r, ref_s, ref_r, scores_of, tol=TOL, tie_band=TIE)
    assert not probs, probs[:5]
    kern, _ = ix.plan(nq, k)
    return kern, s, r


# ---- generator / weights / embeddings: bit-exact ---------------------------------------------------
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("dim", [64, 768, 1024])
def test_synth_rows_bit_exact(rfx, dtype, dim):
    rindex, _ = rfx
    got = stored_to_np(rindex.synth_rows(3, 1000, 257, dim, dtype), dtype)
    ref = osynth.synth_rows(3, 1000, 257, dim, dtype)
    assert got.tobytes() == ref.tobytes()


def test_index_synthetic_rows_match_generator(rfx):
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(11, 300)
    ix.add_synthetic(11, 200)  # continues the row numbering
    got = stored_to_np(ix.read(0, 500), "bf16")
    ref = np.concatenate([osynth.synth_rows(11, 0, 300, 768, "bf16"), osynth.synth_rows(11, 300, 200, 768, "bf16")])
    assert got.tobytes() == ref.tobytes()


def test_embed_weights_bit_exact(rfx):
    _, remb = rfx
    e = remb.Embedder(dim=768, V=4096)
    got = e.weights.cpu().view(torch.int16).numpy().view(np.uint16)
    ref = osynth.f32_to_bf16_bits((oembed.weights_int(4096, 768, e.seed) / 128.0).astype(np.float32))
    assert got.tobytes() == ref.tobytes()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_embed_sample_report_bit_exact(rfx, golden_dir, dtype):
    _, remb = rfx
    text = open(f"{golden_dir}/sample_report.md", encoding="utf-8").read()
    e = remb.Embedder(dim=768)
    chunks, vecs = e.chunk_and_embed(text, dtype, max_tokens=3, overlap=0)
    raw = text.encode()
    spans = textproc.chunk_whitespace(raw, 3, 0)
    assert chunks == [raw[s:t].decode() for s, t in spans]
    csr = textproc.featurize(raw, spans, 4096, e.hash_seed)
    ref = oembed.embed(*csr, 4096, oembed.weights_int(4096, 768, e.seed), dtype)
    assert stored_to_np(vecs, dtype).tobytes() == ref.tobytes()


def test_embed_random_texts_bit_exact(rfx):
    _, remb = rfx
    rng = np.random.default_rng(0)
    words = ["alpha", "Beta", "gamma", "the", "a", "delta-epsilon", "ZETA", "eta9", "über", "naïve", "x", "42"]
    texts = [" ".join(rng.choice(words, size=rng.integers(0, 400))) for _ in range(70)] + ["", "the a an", "!!!"]
    e = remb.Embedder(dim=256, V=1024, seed=5, hash_seed=9)
    vecs = e.embed_texts(texts, "f32").cpu().numpy()
    b = [t.lower().encode() for t in texts]
    raw = b"".join(b)
    offs = np.cumsum([0] + [len(x) for x in b])
    csr = textproc.featurize(raw, list(zip(offs[:-1], offs[1:])), 1024, 9)
    ref = oembed.embed(*csr, 1024, oembed.weights_int(1024, 256, 5), "f32")
    assert vecs.tobytes() == ref.tobytes()
    assert not np.any(vecs[-3:])  # empty / article-only / punctuation-only chunks embed to zero


# ---- search: VALU path (nq <= 8) ----------------------------------------------------------------------
@pytest.mark.parametrize("dtype,dim", [("f32", 768), ("bf16", 768), ("f16", 1024), ("f32", 64), ("bf16", 192)])
@pytest.mark.parametrize("nq", [1, 3, 8])
@pytest.mark.parametrize("k", [1, 5, 10])
def test_search_valu(rfx, dtype, dim, nq, k):
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 20000, dim, dtype, nq, k)
    assert kern == 0


def test_search_cfg2_shape(rfx):
    """BASELINE config 2 shape (100k×768 f32, nq=1, k=10)."""
    rindex, _ = rfx
    kern, s, r = run_search_check(rindex, 100_000, 768, "f32", 1, 10)
    assert kern == 0 and (np.diff(s[0]) <= 0).all()


@pytest.mark.parametrize("k", [16, 33, 64])
def test_search_valu_large_k(rfx, k):
    rindex, _ = rfx
    run_search_check(rindex, 5000, 768, "bf16", 2, k)


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 129])
def test_search_valu_tiny_and_ragged(rfx, n):
    rindex, _ = rfx
    _, s, r = run_search_check(rindex, n, 768, "f32", 1, 10)
    assert (r[0][min(n, 10):] == -1).all() and np.isneginf(s[0][min(n, 10):]).all()


def test_search_empty_index(rfx):
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "f32")
    q = rindex.synth_rows(1, 0, 2, 768, "f32")
    s, r = ix.search(q, 5)
    assert (r.cpu() == -1).all() and torch.isneginf(s.cpu()).all()


@pytest.mark.parametrize("nq", [1, 16])
def test_search_duplicates_tie_break(rfx, nq):
    rindex, _ = rfx
    # duplicate query 0's best row into row 17: the exact tie must rank row 17 first
    rows64 = osynth.to_f64(osynth.synth_rows(7, 0, 10000, 768, "bf16"), "bf16")
    q64 = osynth.to_f64(osynth.synth_rows(8, 0, 1, 768, "bf16"), "bf16")
    top = int(osearch.topk(q64, rows64, 1)[1][0, 0])
    assert top != 17
    _, s, r = run_search_check(rindex, 10000, 768, "bf16", nq, 10, dup=(top, 17))
    assert r[0, 0] == 17 and r[0, 1] == top and s[0, 0] == s[0, 1]


def test_search_tombstones(rfx):
    rindex, _ = rfx
    # tombstone the unfiltered winners: they must never come back
    ix = rindex.DeviceIndex(768, "f32")
    ix.add_synthetic(7, 20000)
    q = rindex.synth_rows(8, 0, 1, 768, "f32")
    _, r0 = ix.search(q, 10)
    dead = r0.cpu().numpy()[0][:4].tolist() + [0, 1, 19999]
    _, s, r = run_search_check(rindex, 20000, 768, "f32", 1, 10, tomb=dead)
    assert not set(dead) & set(r[0].tolist())


# ---- search: MFMA path (batched bf16/f16) ----------------------------------------------------------
def expected_mfma_kernel(nq, k, dim):
    """Mirror of make_layout (rfx_api.hip): 6 = 256-query-stationary, 2 waves/SIMD (d 768, k <= 10, nq > 128),
    8 = 128-query-stationary k-split wave pairs, XCD-paired query groups (d 1024, k <= 10, nq > 64),
    3 = 128-query-stationary (d 768/1024, k <= 16, nq > 64), 2 = 256x256 tiles, 1 = 64-query tiles."""
    if nq > 128 and dim == 768 and k <= 10:
        return 6
    if nq > 64 and dim == 1024 and k <= 10:
        return 8
    if nq > 64 and dim in (768, 1024) and k <= 16:
        return 3
    if nq > 128:
        return 2
    return 1


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("nq", [9, 64, 100, 256, 300])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_search_mfma(rfx, dtype, nq, k):
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 30000, 768, dtype, nq, k)
    assert kern == expected_mfma_kernel(nq, k, 768)


@pytest.mark.parametrize("n", [1, 127, 128, 129, 1000])
def test_search_mfma_ragged(rfx, n):
    rindex, _ = rfx
    kern, s, r = run_search_check(rindex, n, 768, "bf16", 64, 10)
    assert kern == 1


@pytest.mark.parametrize("n,dim", [(1, 768), (255, 768), (256, 768), (257, 768), (70_000, 768), (5000, 64),
                                   (5000, 128), (5000, 192), (3000, 1024), (1000, 1024)])
def test_search_mfma_batched_shapes(rfx, n, dim):
    """nq=256: query-stationary kernel (d 768/1024) or the 256x256 kernel (other d); ragged row
    counts, one tile per block, and D with fewer than 5 K-stages."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, n, dim, "bf16", 256, 10)
    assert kern == expected_mfma_kernel(256, 10, dim)


@pytest.mark.parametrize("k", [1, 4, 5, 8, 16])
def test_search_mfma2_k(rfx, k):
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 50_000, 768, "f16", 200, k)
    assert kern == expected_mfma_kernel(200, k, 768)
    kern, _, _ = run_search_check(rindex, 50_000, 640, "f16", 200, k)
    assert kern == 2


def test_search_mfma2_ties_and_tombstones(rfx):
    rindex, _ = rfx
    rows64 = osynth.to_f64(osynth.synth_rows(7, 0, 20000, 768, "bf16"), "bf16")
    q64 = osynth.to_f64(osynth.synth_rows(8, 0, 1, 768, "bf16"), "bf16")
    top = int(osearch.topk(q64, rows64, 1)[1][0, 0])
    kern, s, r = run_search_check(rindex, 20000, 768, "bf16", 256, 10, dup=(top, 3), tomb=[0, 7, 19999, top + 1])
    assert kern == 6 and r[0, 0] == 3 and r[0, 1] == top


@pytest.mark.parametrize("nq", [65, 128, 129, 384, 512])
def test_search_qstationary_query_groups(rfx, nq):
    """1..4 query groups of 128 resident queries (grid.y), padded last group."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 40_000, 768, "bf16", nq, 10)
    assert kern == expected_mfma_kernel(nq, 10, 768)


@pytest.mark.parametrize("n", [1, 31, 32, 33, 4095, 4097, 100_003])
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_search_mfma4_ragged_rows(rfx, n, dtype):
    """256-query-stationary kernel: 32-row tiles, ragged tails (NaN padding), fewer tiles than CUs."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, n, 768, dtype, 256, 10)
    assert kern == 6


@pytest.mark.parametrize("nq,k", [(129, 10), (255, 1), (256, 4), (257, 10), (512, 5), (600, 10)])
def test_search_mfma4_query_groups(rfx, nq, k):
    """1..3 query groups of 256 (grid.y), padded last group, lane lists of 4 and 10."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 60_000, 768, "bf16", nq, k)
    assert kern == 6


def test_search_mfma4_many_duplicates(rfx):
    """Twelve copies of the best row for query 0 (more than k): the lowest row ids win, in order."""
    rindex, _ = rfx
    n = 50_000
    rows64 = osynth.to_f64(osynth.synth_rows(7, 0, n, 768, "bf16"), "bf16")
    q64 = osynth.to_f64(osynth.synth_rows(8, 0, 1, 768, "bf16"), "bf16")
    top = int(osearch.topk(q64, rows64, 1)[1][0, 0])
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(7, n)
    allr = ix.read(0, n)
    dst = [5, 40, 41, 999, 1000, 1001, 20_000, 33_333, 40_001, 45_000, 49_998, 49_999]
    for d in dst:
        allr[d] = allr[top]
    ix2 = rindex.DeviceIndex(768, "bf16")
    ix2.add(allr)
    q = rindex.synth_rows(8, 0, 256, 768, "bf16")
    s, r = ix2.search(q, 10)
    assert ix2.plan(256, 10)[0] == 6
    want = sorted(dst + [top])[:10]
    assert r[0].cpu().tolist() == want
    assert float(s[0, 0]) == float(s[0, 9])


# ---- kernel 9 (f32 stores, 16 < nq): f32 MFMA, 32 resident queries per wave, one wave per SIMD ------
@pytest.mark.parametrize("n", [1, 63, 64, 65, 8191, 30_001])
def test_search_f32_batched_ragged_rows(rfx, n):
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, n, 768, "f32", 256, 10)
    assert kern == 9


@pytest.mark.parametrize("nq,k", [(16, 10), (17, 10), (64, 4), (128, 1), (129, 10), (300, 5)])
def test_search_f32_batched_query_groups(rfx, nq, k):
    """nq <= 16 stays on the VALU slices; above, 1..3 query groups of 128, lane lists of 4 and 10."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 40_000, 768, "f32", nq, k)
    assert kern == (9 if nq > 16 else 0)


def test_search_f32_batched_ties_and_tombstones(rfx):
    rindex, _ = rfx
    rows64 = osynth.to_f64(osynth.synth_rows(7, 0, 20000, 768, "f32"), "f32")
    q64 = osynth.to_f64(osynth.synth_rows(8, 0, 1, 768, "f32"), "f32")
    top = int(osearch.topk(q64, rows64, 1)[1][0, 0])
    kern, s, r = run_search_check(rindex, 20000, 768, "f32", 64, 10, dup=(top, 3), tomb=[0, 7, 19999, top + 1])
    assert kern == 9 and r[0, 0] == 3 and r[0, 1] == top


def test_f32_batched_matches_valu_slices(rfx):
    """The same 64 queries through kernel 9 and through the VALU scan in 8-query slices."""
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "f32")
    ix.add_synthetic(21, 100_000)
    q = rindex.synth_rows(22, 0, 64, 768, "f32")
    s1, r1 = ix.search(q, 10)
    assert ix.plan(64, 10)[0] == 9
    parts = [ix.search(q[i:i + 8], 10) for i in range(0, 64, 8)]
    s2 = torch.cat([p[0] for p in parts]).cpu().numpy()
    r2 = torch.cat([p[1] for p in parts]).cpu().numpy()
    s1, r1 = s1.cpu().numpy(), r1.cpu().numpy()
    assert np.abs(s1 - s2).max() <= 2 * TOL
    for qi, ki in zip(*np.nonzero(r1 != r2)):
        assert abs(s1[qi, ki] - s2[qi, ki]) <= 2 * TIE


def test_search_mfma_dim1024(rfx):
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 20000, 1024, "f16", 128, 10)
    assert kern == 8


# ---- kernel 8 (d = 1024, config 4): 64-row tiles, k-split wave pairs, query groups paired on one XCD ----
@pytest.mark.parametrize("n", [1, 63, 64, 65, 127, 129, 8191, 16_385, 100_003])
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_search_d1024_ragged_rows(rfx, n, dtype):
    """Ragged 64-row tails (NaN padding), fewer tiles than ranges (unpaired grid), paired grid."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, n, 1024, dtype, 256, 10)
    assert kern == 8


@pytest.mark.parametrize("nq,k", [(65, 10), (128, 1), (129, 4), (200, 10), (256, 10), (300, 5), (512, 10)])
def test_search_d1024_query_groups(rfx, nq, k):
    """1..4 query groups of 128 (padded last group), lane lists of 4 and 10."""
    rindex, _ = rfx
    kern, _, _ = run_search_check(rindex, 60_000, 1024, "f16", nq, k)
    assert kern == 8


def test_search_d1024_ties_and_tombstones(rfx):
    rindex, _ = rfx
    rows64 = osynth.to_f64(osynth.synth_rows(7, 0, 30000, 1024, "f16"), "f16")
    q64 = osynth.to_f64(osynth.synth_rows(8, 0, 1, 1024, "f16"), "f16")
    top = int(osearch.topk(q64, rows64, 1)[1][0, 0])
    kern, s, r = run_search_check(rindex, 30000, 1024, "f16", 256, 10, dup=(top, 3), tomb=[0, 7, 29999, top + 1])
    assert kern == 8 and r[0, 0] == 3 and r[0, 1] == top


def test_search_mfma_ties_and_tombstones(rfx):
    rindex, _ = rfx
    run_search_check(rindex, 20000, 768, "bf16", 32, 10, dup=(1234, 5), tomb=[0, 7, 1234, 19999])


def test_mfma_matches_valu_path(rfx):
    """Same queries through both kernels: identical row lists up to the tie band."""
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(21, 200_000)
    q = rindex.synth_rows(22, 0, 64, 768, "bf16")
    s1, r1 = ix.search(q, 10)
    assert ix.plan(64, 10)[0] == 1
    parts = [ix.search(q[i:i + 8], 10) for i in range(0, 64, 8)]
    s2 = torch.cat([p[0] for p in parts]).cpu().numpy()
    r2 = torch.cat([p[1] for p in parts]).cpu().numpy()
    s1, r1 = s1.cpu().numpy(), r1.cpu().numpy()
    mism = (r1 != r2)
    assert np.abs(s1 - s2).max() < 2 * TOL
    # any order difference must be a near-tie
    for qi, ki in zip(*np.nonzero(mism)):
        assert abs(s1[qi, ki] - s2[qi, ki]) <= 2 * TIE


def test_self_retrieval_property(rfx):
    """Size-independent property: a stored row used as the query ranks itself first (score 1)."""
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(5, 300_000)
    rows = [0, 1, 77_777, 299_999] + list(range(1000, 1000 + 60))
    q = torch.cat([ix.read(r, 1) for r in rows])
    s, r = ix.search(q, 10)
    r = r.cpu().numpy()
    assert (r[:, 0] == np.array(rows)).all()
    assert (np.abs(s.cpu().numpy()[:, 0] - 1.0) < 1e-2).all()


def test_merge_shards_equals_whole(rfx):
    """Row-sharded search + cross-shard merge == unsharded search (the multi-GPU exchange step)."""
    rindex, _ = rfx
    whole = rindex.DeviceIndex(768, "bf16")
    whole.add_synthetic(31, 40_000)
    shards = []
    for i in range(4):
        sh = rindex.DeviceIndex(768, "bf16")
        sh.add(whole.read(i * 10_000, 10_000))
        shards.append(sh)
    q = rindex.synth_rows(32, 0, 40, 768, "bf16")
    s0, r0 = whole.search(q, 10)
    parts = [sh.search(q, 10) for sh in shards]
    cs = torch.cat([p[0] for p in parts], dim=1)
    cr = torch.cat([p[1] + i * 10_000 for i, p in enumerate(parts)], dim=1)
    s1, r1 = rindex.topk_merge(cs, cr, 10)
    assert torch.equal(r0.cpu(), r1.cpu())
    assert torch.equal(s0.cpu(), s1.cpu())


def test_save_load_roundtrip(rfx, tmp_path):
    rindex, _ = rfx
    ix = rindex.DeviceIndex(768, "f16")
    ix.add_synthetic(3, 5000)
    ix.tombstone([10, 20])
    p = str(tmp_path / "x.rfx")
    ix.save(p)
    iy = rindex.DeviceIndex.load(p)
    assert iy.rows == 5000 and iy.live_rows == 4998 and iy.dtype == "f16"
    q = rindex.synth_rows(4, 0, 3, 768, "f16")
    a, b = ix.search(q, 10), iy.search(q, 10)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])


# ---- the adapter end to end on the GPU (config 1 plumbing) -------------------------------------------
def test_adapter_cfg1_end_to_end(rfx, golden_dir, tmp_path, monkeypatch):
    import json

    from rfx import store as rstore
    from rfx.adapter import LocalGpuRag
    from rfx.retriever import GpuRetriever

    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path)))
    rag = LocalGpuRag(GpuRetriever(dtype="f32"), top_k=5)
    st = rag.create_store("demo")
    assert st.startswith("fileSearchStores/")
    up = rag.upload_file(st, f"{golden_dir}/sample_report.md", display_name="sample-report.md",
                         chunking_config={"white_space_config": {"max_tokens_per_chunk": 3, "max_overlap_tokens": 0}})
    assert up.operation_name.startswith("operations/") and up.file_id.startswith("files/")
    assert rag.op_status(up.operation_name)["done"] is True
    fx = json.load(open(f"{golden_dir}/cfg1_sample_report.json"))
    for case in fx["queries"]:
        q = case["question"]
        chunks = list(rag.ask_stream(contents=[{"role": "user", "parts": [{"text": q}]}], store_names=[st],
                                     metadata_filter=None, model="gemini-2.5-flash"))
        assert len(chunks) == 2 and chunks[0].text == f"[mock-mode] {q}" and chunks[0].candidates is None
        cits = rag.extract_citations_from_response(chunks[1])
        assert [c["index"] for c in cits] == list(range(len(cits)))
        assert [c["snippet"] for c in cits] == case["snippets"]
        gc = chunks[1].candidates[0].grounding_metadata.grounding_chunks
        rows = [g.retrieved_context.row for g in gc]
        assert rows == case["rows"]
        assert np.allclose([g.retrieved_context.score for g in gc], case["scores"], atol=TOL, rtol=0)
    # delete the document: its chunks disappear from retrieval
    rag.delete_document_from_store(st, 1, "sample-report.md", file_id=up.file_id)
    assert rag.retrieve("mock-mode document assistant", [st]) == []
    rag.delete_store(st)


def test_concurrent_retrieval_is_batched_and_equals_sequential(rfx, golden_dir, tmp_path):
    """Micro-batching (rfx.batcher): 32 threads asking at once share GPU batches (fewer batches
    than questions) and each gets the rows it gets alone."""
    import threading

    from rfx import retriever as rret
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path)))
    ret = GpuRetriever(dtype="bf16")
    st = ret.create_store("demo")
    text = open(f"{golden_dir}/sample_report.md").read()
    ret.add_document(st, text * 20, "doc", {"white_space_config": {"max_tokens_per_chunk": 5, "max_overlap_tokens": 1}})
    words = text.split()
    questions = [" ".join(words[i:i + 4]) for i in range(0, 4 * 32, 4)]
    ret.batching = False
    solo = [[(h.row, h.score) for h in ret.search([st], q, 5)] for q in questions]
    ret.batching = True
    out = [None] * len(questions)
    gate = threading.Barrier(len(questions))

    def ask(i):
        gate.wait()
        out[i] = [(h.row, h.score) for h in ret.search([st], questions[i], 5)]

    th = [threading.Thread(target=ask, args=(i,)) for i in range(len(questions))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    # same rows in the same order; scores within the parity tolerance (a batch of 32 runs the MFMA
    # scan, a lone question the VALU scan: different f32 summation order)
    assert [[r for r, _ in o] for o in out] == [[r for r, _ in o] for o in solo]
    assert max(abs(a[1] - b[1]) for o, so in zip(out, solo) for a, b in zip(o, so)) <= TOL
    b = [v for k, v in rret._BATCHERS.items() if k[0] == st][0]
    assert b.items == len(questions) and b.batches < len(questions)
