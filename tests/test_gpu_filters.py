"""GPU parity of metadata-filtered search (rfx_search_masked / rfx_scan_topk_masked, SURVEY §8f
item 4): every scan kernel with a row mask returns what the oracle returns over the allowed rows
only (excluded rows = NaN, the tombstone rule), under the parity bars of test_gpu_parity.py."""
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
    import rfx.index as rindex
    return rindex


def mask_words(allowed: np.ndarray) -> np.ndarray:
    n = len(allowed)
    pad = np.zeros(max(1, (n + 31) // 32) * 32, dtype=np.uint8)
    pad[:n] = allowed
    return np.packbits(pad, bitorder="little").view("<u4").view(np.int32)


def check_masked(rindex, n, dim, dtype, nq, k, allowed, seed=11, qseed=12, tomb=None, expect_kernel=None):
    ix = rindex.DeviceIndex(dim, dtype)
    ix.add_synthetic(seed, n)
    rows64 = osynth.to_f64(osynth.synth_rows(seed, 0, n, dim, dtype), dtype)
    if tomb is not None:
        ix.tombstone(tomb)
        rows64[np.asarray(tomb)] = np.nan
    ref_rows = np.where(allowed[:, None], rows64, np.nan)
    q = rindex.synth_rows(qseed, 0, nq, dim, dtype)
    q64 = osynth.to_f64(osynth.synth_rows(qseed, 0, nq, dim, dtype), dtype)
    m = torch.from_numpy(mask_words(allowed)).cuda()
    s, r = ix.search(q, k, row_mask=m)
    torch.cuda.synchronize()
    s, r = s.cpu().numpy(), r.cpu().numpy()
    ref_s, ref_r = osearch.topk(q64, ref_rows, k)
    probs = osearch.check_topk(s, r, ref_s, ref_r, lambda qi, rows: ref_rows[rows] @ q64[qi], tol=TOL, tie_band=TIE)
    assert not probs, probs[:5]
    live = r[r >= 0]
    assert allowed[live].all(), "a masked-out row was returned"
    if expect_kernel is not None:
        assert ix.plan(nq, k)[0] == expect_kernel
    return ix, s, r


# (dim, dtype, nq, k, kernel): every production kernel of make_layout
KERNEL_CASES = [
    (768, "f32", 1, 10, 0),    # VALU, one query
    (768, "bf16", 6, 5, 0),    # VALU, 8-query slices
    (768, "bf16", 40, 10, 1),  # 64-query MFMA tiles
    (768, "f16", 100, 16, 3),  # 128-query-stationary
    (1024, "f16", 200, 10, 8),  # d-1024 kernel (config 4)
    (1024, "f16", 200, 16, 3),
    (256, "bf16", 200, 10, 2),  # 256x256 tiles, other d
    (768, "f32", 100, 10, 9),   # f32 stores, batched (kernel 9)
    (768, "bf16", 256, 10, 6),  # the config-3 kernel
    (768, "f16", 300, 4, 6),    # kernel 6, KL 4, two query groups
    (1024, "bf16", 256, 4, 8),  # kernel 8, KL 4
    (768, "f32", 40, 3, 9),     # kernel 9, KL 4, one partial query group
]


@pytest.mark.parametrize("dim,dtype,nq,k,kern", KERNEL_CASES)
@pytest.mark.parametrize("density", [0.3, 0.002])
def test_masked_search_every_kernel(rindex, dim, dtype, nq, k, kern, density):
    n = 20_011  # ragged: not a multiple of any tile
    rng = np.random.default_rng(int(density * 1000) + nq)
    allowed = rng.random(n) < density
    check_masked(rindex, n, dim, dtype, nq, k, allowed, expect_kernel=kern)


@pytest.mark.parametrize("n", [19_973, 65, 100])
def test_masked_d1024_odd_mask_words(rindex, n):
    """The d-1024 kernel's 64-row tiles span two mask words: the last tile's second word may lie past the
    (rows + 31) / 32 words of the mask (n = 19,973: 625 words, 313 tiles)."""
    allowed = np.random.default_rng(n).random(n) < 0.5
    allowed[-1] = True
    check_masked(rindex, n, 1024, "bf16", 256, 10, allowed, expect_kernel=8)


@pytest.mark.parametrize("dim,dtype,nq,k,kern", [KERNEL_CASES[0], KERNEL_CASES[2], KERNEL_CASES[7], KERNEL_CASES[8]])
def test_masked_search_ranges_and_tombstones(rindex, dim, dtype, nq, k, kern):
    # file-shaped masks (contiguous ranges, as LocalStore.row_mask builds them) plus tombstones
    n = 50_000
    allowed = np.zeros(n, dtype=bool)
    for a, b in ((0, 7), (31, 33), (1000, 1337), (40_000, 49_999)):
        allowed[a:b] = True
    check_masked(rindex, n, dim, dtype, nq, k, allowed, tomb=list(range(1010, 1100)) + [40_000], expect_kernel=kern)


@pytest.mark.parametrize("nq", [1, 40, 256])
def test_mask_all_and_none(rindex, nq):
    n, dim, dtype, k = 9_000, 768, "bf16", 10
    ix, s, r = check_masked(rindex, n, dim, dtype, nq, k, np.ones(n, dtype=bool))
    s0, r0 = ix.search(rindex.synth_rows(12, 0, nq, dim, dtype), k)
    assert np.array_equal(r, r0.cpu().numpy()) and np.array_equal(s, s0.cpu().numpy())
    _, s, r = check_masked(rindex, n, dim, dtype, nq, k, np.zeros(n, dtype=bool))
    assert (r == -1).all() and np.isneginf(s).all()


def test_masked_scan_then_merge(rindex):
    # the two halves (rfx_scan_topk_masked + merge) equal the fused masked search
    n, dim, dtype, nq, k = 30_000, 768, "bf16", 256, 10
    allowed = np.random.default_rng(5).random(n) < 0.1
    ix, s, r = check_masked(rindex, n, dim, dtype, nq, k, allowed)
    m = torch.from_numpy(mask_words(allowed)).cuda()
    q = rindex.synth_rows(12, 0, nq, dim, dtype)
    cs, cr = ix.scan(q, k, row_mask=m)
    ms, mr = rindex.rescore_topk(ix, q, *rindex.topk_merge(cs, cr, k))  # the search's score rule
    assert np.array_equal(mr.cpu().numpy(), r) and np.array_equal(ms.cpu().numpy(), s)


def test_mask_validation(rindex):
    ix = rindex.DeviceIndex(768, "bf16")
    ix.add_synthetic(1, 100)
    q = rindex.synth_rows(2, 0, 4, 768, "bf16")
    with pytest.raises(ValueError):
        ix.search(q, 5, row_mask=torch.zeros(3, dtype=torch.int32, device="cuda"))  # needs 4 words
    with pytest.raises(ValueError):
        ix.search(q, 5, row_mask=torch.zeros(4, dtype=torch.int64, device="cuda"))


def test_retriever_filter_end_to_end(rindex, tmp_path):
    # LocalGpuRag over GpuRetriever: upload metadata -> filter -> row mask -> masked scan
    from rfx.adapter import LocalGpuRag
    from rfx.retriever import GpuRetriever
    from rfx.store import StoreRegistry, set_registry

    set_registry(StoreRegistry(root=str(tmp_path / "stores")))
    rag = LocalGpuRag(GpuRetriever(dtype="bf16"), top_k=5)
    st = rag.create_store("tenants")
    for tenant, words in (("acme", "alpha beta gamma delta " * 8), ("globex", "alpha beta epsilon zeta " * 8)):
        p = tmp_path / f"{tenant}.txt"
        p.write_text(words)
        rag.upload_file(st, str(p), display_name=f"{tenant}.txt",
                        custom_metadata=[{"key": "tenant", "string_value": tenant}],
                        chunking_config={"white_space_config": {"max_tokens_per_chunk": 4, "max_overlap_tokens": 0}})

    def titles(filt):
        r = rag.ask(contents="alpha beta", store_names=[st], metadata_filter=filt, model="m", top_k=20)
        return [c["title"] for c in rag.extract_citations_from_response(r)]

    everything = titles(None)
    assert set(everything) == {"acme.txt", "globex.txt"}
    assert titles({"tenant": "acme"}) == [t for t in everything if t == "acme.txt"]
    assert titles({"tenant": ["globex"]}) == [t for t in everything if t == "globex.txt"]
    assert titles({"tenant": "initech"}) == []


def test_filter_survives_store_reload(rindex, tmp_path):
    # upload metadata is persisted with the store (manifest.json): another process (a fresh
    # registry on the same directory, as the API workers load what the ingestion worker wrote)
    # applies the same filter
    from rfx.adapter import LocalGpuRag
    from rfx.retriever import GpuRetriever
    from rfx.store import StoreRegistry, set_registry

    root = str(tmp_path / "stores")
    set_registry(StoreRegistry(root=root))
    rag = LocalGpuRag(GpuRetriever(dtype="bf16"), top_k=5)
    st = rag.create_store("tenants")
    for tenant, words in (("acme", "alpha beta gamma delta " * 8), ("globex", "alpha beta epsilon zeta " * 8)):
        p = tmp_path / f"{tenant}.txt"
        p.write_text(words)
        rag.upload_file(st, str(p), display_name=f"{tenant}.txt",
                        custom_metadata=[{"key": "tenant", "string_value": tenant}],
                        chunking_config={"white_space_config": {"max_tokens_per_chunk": 4, "max_overlap_tokens": 0}})
    ask = lambda r: [c["title"] for c in r.extract_citations_from_response(
        r.ask(contents="alpha beta", store_names=[st], metadata_filter={"tenant": "globex"}, model="m", top_k=20))]
    before = ask(rag)
    set_registry(StoreRegistry(root=root))  # fresh process view: loads manifest + index from disk
    after = ask(LocalGpuRag(GpuRetriever(dtype="bf16"), top_k=5))
    assert before == after and set(after) == {"globex.txt"}
