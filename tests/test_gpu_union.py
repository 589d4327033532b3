"""GPU: a question over several stores is ONE scan of their union (rfx.union.UnionView behind
GpuRetriever.search; the file-search tool's store list, gemini_rag.py:463-469).  The hits equal
the per-store path's (one scan per store + host merge by score desc, store order, row asc) exactly,
with and without a metadata filter, after growth and deletion, and the union path calls the
device search once per batch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DOCS = [("alpha beta gamma delta epsilon " * 30, {"tenant": "acme"}),
        ("zeta eta theta iota kappa lambda " * 25, {"tenant": "globex"}),
        ("mock mode document assistant retrieval citations " * 20, {"tenant": "acme"}),
        ("hbm bandwidth roofline matrix cores wavefront lds " * 23, None),
        ("alpha theta roofline citations kappa " * 17, {"tenant": "globex"})]
QUESTIONS = ["alpha gamma", "theta kappa lambda", "document retrieval", "roofline lds", "beta zeta assistant"]
WS = {"white_space_config": {"max_tokens_per_chunk": 4, "max_overlap_tokens": 1}}


def _hits(ret, names, q, k, filt=None):
    return [(h.score, h.store, h.row, h.file_id, h.text) for h in ret.search(names, q, k, metadata_filter=filt)]


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_union_equals_per_store(tmp_path, dtype, monkeypatch):
    from rfx import store as rstore
    from rfx.index import DeviceIndex
    from rfx.retriever import GpuRetriever

    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype=dtype)
    names = [ret.create_store(f"s{i}") for i in range(3)]
    fids = []
    for i, (t, m) in enumerate(DOCS):
        fids.append(ret.add_document(names[i % 3], t, f"doc{i}", WS, m)[0])
    ret.batching = False  # the single-question path; the batched one is below

    calls = []
    orig = DeviceIndex.search
    monkeypatch.setattr(DeviceIndex, "search", lambda self, *a, **kw: calls.append(self) or orig(self, *a, **kw))

    def same(filt=None):
        for q in QUESTIONS:
            for k in (1, 5, 10, 33):
                ret.union = True
                calls.clear()
                a = _hits(ret, names, q, k, filt)
                # one device search per question; none when the filter matches no file of any store
                want = 0 if filt == {"tenant": "nobody"} else 1
                assert ret.last_path == "union" and len(calls) == want, (ret.last_path, len(calls))
                ret.union = False
                b = _hits(ret, names, q, k, filt)
                assert ret.last_path == "per-store"
                assert a == b, (q, k, filt)

    same()
    same({"tenant": "acme"})
    same({"tenant": "nobody"})
    # growth and deletion: the view is rebuilt from the members' new committed state
    ret.add_document(names[1], "nu xi omicron pi rho sigma alpha " * 12, "late", WS, {"tenant": "acme"})
    ret.delete_file(names[0], fids[0])
    same()
    same({"tenant": "globex"})
    # two stores, listed in the other order: store order follows the list
    ret.union = True
    a = _hits(ret, [names[2], names[0]], "alpha roofline", 10)
    ret.union = False
    assert a == _hits(ret, [names[2], names[0]], "alpha roofline", 10)


def test_union_batched_questions(tmp_path):
    """Concurrent questions over the same store list share one union launch per batch."""
    import threading

    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype="bf16")
    names = [ret.create_store(f"b{i}") for i in range(3)]
    for i, (t, m) in enumerate(DOCS):
        ret.add_document(names[i % 3], t, f"doc{i}", WS, m)
    qs = [f"{w} {v}" for w in ("alpha", "theta", "roofline", "document") for v in ("gamma", "kappa", "lds", "cores")]
    lone = {}
    ret.batching = False
    for q in qs:
        lone[q] = _hits(ret, names, q, 7)
    ret.batching = True
    got, errs = {}, []

    def worker(q):
        try:
            got[q] = _hits(ret, names, q, 7)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=worker, args=(q,)) for q in qs]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not errs and set(got) == set(lone)
    # a batch runs the batched kernels (a lone question the VALU scan): the same rows, scores within
    # the parity tolerance (1e-5), order free only inside the 2e-6 tie band
    for q in qs:
        a, b = got[q], lone[q]
        assert len(a) == len(b)
        assert all(abs(x[0] - y[0]) <= 1e-5 for x, y in zip(a, b)), q
        if all(b[i][0] - b[i + 1][0] > 2e-6 for i in range(len(b) - 1)):
            assert [x[1:] for x in a] == [y[1:] for y in b], q
    torch.cuda.synchronize()
