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


def _synth_store(reg, name, n, seed, files=4):
    """A store of n synthetic bf16 rows in `files` uploads (LocalStore.add_document with device rows)."""
    from rfx.index import synth_rows
    st = reg.create(name, 768, "bf16")
    per = -(-n // files)
    fids = []
    for f in range(files):
        m = min(per, n - f * per)
        vecs = synth_rows(seed, f * per, m, 768, "bf16")
        fids.append(st.add_document([f"{name}-{f}-{i}" for i in range(m)], vecs, f"{name}-{f}.md",
                                    {"part": f})[0])
    return st, fids


@pytest.mark.parametrize("mode", ["map", "copy"])
def test_union_follows_member_appends_in_place(tmp_path, mode, monkeypatch):
    """an upload to one member of a 3-store union of > 1M rows costs O(appended
    rows) — the copying view copies only the new rows into that member's headroom and re-applies new
    tombstones; the zero-copy view (the default) copies no row at all: its rows are the
    members' memory, mapped back to back, and its own device bytes are the tile records (16 B per 32
    rows) and stats.  Hits stay identical to the per-store path either way."""
    import time
    monkeypatch.setenv("RFX_UNION_COPY", "1" if mode == "copy" else "0")

    from rfx import retriever as rret
    from rfx import store as rstore
    from rfx.index import synth_rows
    from rfx.retriever import GpuRetriever

    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype="bf16")
    ret.batching = False
    stores = [_synth_store(reg, f"u{i}", 350_000 + 1000 * i, 40 + i) for i in range(3)]
    names = [st.name for st, _ in stores]

    def check(q):
        ret.union = True
        a = _hits(ret, names, q, 10)
        assert ret.last_path == "union"
        ret.union = False
        assert a == _hits(ret, names, q, 10)
        return a

    t0 = time.perf_counter()
    check("alpha gamma")
    t_build = time.perf_counter() - t0
    key = (tuple(names), id(reg))
    view = rret._UNIONS[key]
    assert view.mapped == (mode == "map")
    n_rows = sum(st.index.rows for st, _ in stores)
    if mode == "map":
        assert view.rows_copied == 0 and n_rows >= 1_000_000
        # the view's own device bytes: the tile records and stats of the int8 copy, nothing of the rows
        assert view.nbytes == (sum(view.regions) // 32 * 16 + 256 if view.screened else 0)
        assert view.nbytes * 1000 < n_rows * 768 * 2
    else:
        assert view.rows_copied == n_rows >= 1_000_000
    st1 = stores[1][0]
    cap1 = st1.index.capacity
    st1.add_document([f"late-{i}" for i in range(1500)], synth_rows(99, 0, 1500, 768, "bf16"), "late.md")
    t0 = time.perf_counter()
    check("theta kappa")
    t_follow = time.perf_counter() - t0
    grown = st1.index.capacity != cap1  # (a member that outgrows its capacity moves its memory: a new view)
    if not grown:
        assert rret._UNIONS[key] is view
    view = rret._UNIONS[key]
    assert view.rows_copied == (0 if mode == "map" else sum(st.index.rows for st, _ in stores))
    assert view.rows[1] == st1.index.rows
    copied = view.rows_copied
    stores[2][0].delete_file(stores[2][1][1])
    check("document retrieval")
    assert rret._UNIONS[key] is view and view.rows_copied == copied  # tombstones only: no rows copied
    print(f"union ({mode}) of {sum(view.rows)} rows: build+search {t_build * 1e3:.1f} ms, follow 1500 appended "
          f"rows + search {t_follow * 1e3:.1f} ms")
    if mode == "copy":
        assert t_follow < t_build


def test_union_cache_stays_within_its_byte_budget(tmp_path, monkeypatch):
    """The view cache is bounded in bytes (RFX_UNION_MAX_BYTES, LRU), not by a count; a list whose view
    alone exceeds the budget takes the per-store path.  (Copying views: a zero-copy view holds only its tile
    records, which no realistic budget excludes.)"""
    monkeypatch.setenv("RFX_UNION_COPY", "1")
    from rfx import retriever as rret
    from rfx import store as rstore
    from rfx import union as runion
    from rfx.retriever import GpuRetriever

    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype="bf16")
    ret.batching = False
    names = [ret.create_store(f"c{i}") for i in range(4)]
    for i, (t, m) in enumerate(DOCS):
        ret.add_document(names[i % 4], t, f"doc{i}", WS, m)
    pair = runion.planned_bytes([reg.get(names[0]), reg.get(names[1])])
    monkeypatch.setenv("RFX_UNION_MAX_BYTES", str(int(pair * 2.5)))
    budget = rret.union_budget()
    lists = [[names[0], names[1]], [names[2], names[3]], [names[0], names[2]], [names[1], names[3]],
             [names[0], names[1]]]
    for lst in lists:
        ret.union = True
        a = _hits(ret, lst, "alpha theta", 6)
        assert ret.last_path == "union"
        ret.union = False
        assert a == _hits(ret, lst, "alpha theta", 6)
        mine = [v for k, v in rret._UNIONS.items() if k[1] == id(reg)]
        assert rret._UNION_BYTES[0] <= budget and sum(v.nbytes for v in mine) <= budget
    monkeypatch.setenv("RFX_UNION_MAX_BYTES", str(pair // 2))  # no view fits: per-store path, same hits
    ret.union = True
    a = _hits(ret, names[:3], "roofline lds", 8)
    assert ret.last_path == "per-store"


def test_single_store_question_while_a_union_builds(tmp_path, monkeypatch):
    """a union view is built outside the process-wide _STATE_LOCK. A thread builds the
    view of a 1,000,000-row store and a small one (held inside the build, between its first member copy
    and the rest); meanwhile a single-store question through the same retriever completes."""
    import threading

    from rfx import retriever as rret
    from rfx import store as rstore
    from rfx import union as runion
    from rfx.index import synth_rows
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_UNION_COPY", "1")  # the copying view (its member copy is what the test holds)
    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype="bf16")
    ret.batching = False
    small, big = ret.create_store("small"), ret.create_store("big")
    for t, m in DOCS:
        ret.add_document(small, t, "d", WS, m)
    n_big = 1_000_000
    reg.get(big).add_document(["c"] * n_big, synth_rows(5, 0, n_big, 768, "bf16", device=0), "bulk")
    want = _hits(ret, [small], "alpha gamma", 5)
    started, release = threading.Event(), threading.Event()
    orig = runion.UnionView._copy

    def held_copy(self, *a, **kw):  # the first member copy of the build waits for the question below
        if not started.is_set():
            started.set()
            assert release.wait(60)
        return orig(self, *a, **kw)

    monkeypatch.setattr(runion.UnionView, "_copy", held_copy)
    out = {}
    stores = [reg.get(big), reg.get(small)]
    t = threading.Thread(target=lambda: out.setdefault("v", ret._union_view([big, small], stores)))
    t.start()
    try:
        assert started.wait(60)
        got = _hits(ret, [small], "alpha gamma", 5)  # the build is in progress (and blocked)
        assert got == want and t.is_alive()
    finally:
        release.set()
        t.join(120)
    v = out["v"]
    assert v.rows == [n_big, reg.get(small).index.rows]
    rret._release_union(v)


def test_zero_copy_union_holds_no_copy_of_the_members(tmp_path, monkeypatch):
    """a question over several stores reads the members in place.  The zero-copy view maps
    the members' rows and int8 copies back to back (rfx_union_create, HIP virtual memory): building it takes
    no device memory beyond its tile records (16 B per 32 rows) and stats, its answers equal the per-store
    path's bit for bit (batched, through the 2-wave kernel 10; and a lone question, kernel 11), and the
    members' appends and tombstones show through after a refresh of the records alone."""
    import numpy as np

    from rfx import retriever as rret
    from rfx import store as rstore
    from rfx.index import synth_rows
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_UNION_COPY", "0")
    monkeypatch.setenv("RFX_SCREEN", "1")
    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    ret = GpuRetriever(registry=reg, dtype="bf16")
    made = [_synth_store(reg, f"z{i}", 600_000 + 7_777 * i, 70 + i) for i in range(3)]
    stores = [st for st, _ in made]
    assert all(st._screen_on is True for st in stores)
    names = [st.name for st in stores]
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    view = ret._union_view(names, stores)
    torch.cuda.synchronize()
    used = free0 - torch.cuda.mem_get_info()[0]
    rows_bytes = sum(st.index.capacity for st in stores) * 768 * 3  # bf16 rows + int8 codes
    assert view.mapped and view.screened and view.rows_copied == 0
    assert view.nbytes == sum(view.regions) // 32 * 16 + 256
    # (the allocator's granules: at most a few MiB, against the 5+ GB a copy would take)
    assert used <= view.nbytes + (64 << 20) and used * 100 < rows_bytes, (used, rows_bytes)
    rret._release_union(view)

    def compare(k, nq):
        qs = [synth_rows(200 + i, 0, 1, 768, "bf16") for i in range(nq)]
        q = torch.cat(qs)
        v = ret._union_view(names, stores)
        try:
            s_u, r_u = v.index.search(q, k)
            si, ri = v.locate(r_u.cpu().numpy())
        finally:
            rret._release_union(v)
        # the per-store path: each member searched alone, merged by (score desc, store order, row asc)
        per = [st.index.search(q, k) for st in stores]
        s_u = s_u.cpu().numpy()
        for qi in range(nq):
            cand = []
            for m, (s, r) in enumerate(per):
                s, r = s[qi].cpu().numpy(), r[qi].cpu().numpy()
                cand += [(-float(s[j]), m, int(r[j])) for j in range(k) if r[j] >= 0]
            cand.sort()
            want = cand[:k]
            got = [(-float(s_u[qi, j]), int(si[qi, j]), int(ri[qi, j])) for j in range(k)]
            assert got == want, (qi, got[:3], want[:3])

    compare(10, 32)  # a micro-batch: the 2-wave kernel 10 on the view
    compare(10, 1)   # a lone question: kernel 11 on the view
    # appends within a member's capacity and a deletion: the view follows without a copy
    st1 = stores[1]
    cap = st1.index.capacity
    n_new = min(2_000, cap - st1.index.rows)
    if n_new > 0:
        st1.add_document([f"late-{i}" for i in range(n_new)], synth_rows(99, 0, n_new, 768, "bf16"), "late.md")
    assert stores[2].delete_file(made[2][1][1])
    v2 = ret._union_view(names, stores)
    assert v2 is view and v2.rows_copied == 0 and np.array_equal(v2.rows, [st.index.rows for st in stores])
    rret._release_union(v2)
    compare(10, 32)
    rret._purge_batchers(names[0])
    for st in stores:
        reg.drop(st.name)
