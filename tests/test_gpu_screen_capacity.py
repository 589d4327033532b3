"""GPU: the capacity guard of the int8 copy (VERDICT r3 missing #2 / next #3).

rfx_index_screen refuses a copy that does not fit (RFX_ECAPACITY: free device memory minus a reserve,
or RFX_SCREEN_MAX_BYTES) and the index stays exact; an append that outgrows the copy drops it and
succeeds; a store upload past the cap commits, does not raise, and answers with the exact plan.
Reference seam: ingestion.py:311-339 (what a raise after the commit would do to the document)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_enable_screen_past_the_cap_stays_exact(monkeypatch):
    from rfx._lib import RfxCapacityError
    from rfx.index import DeviceIndex, synth_rows

    ix = DeviceIndex(768, "bf16", 0)
    ix.add_synthetic(1, 5000)
    q = synth_rows(2, 0, 256, 768, "bf16")
    ref = ix.search(q, 10)
    monkeypatch.setenv("RFX_SCREEN_MAX_BYTES", "1000")
    with pytest.raises(RfxCapacityError):
        ix.enable_screen(1)
    assert ix.screen_state() == (0, 0, False) and ix.search_plan(256, 10) == 6
    got = ix.search(q, 10)
    assert torch.equal(got[1], ref[1]) and torch.equal(got[0], ref[0])
    ix.close()


def test_append_that_outgrows_the_copy_drops_it(monkeypatch):
    from rfx.index import DeviceIndex, synth_rows

    ix = DeviceIndex(768, "bf16", 0)
    ix.add_synthetic(3, 5000)
    ix.enable_screen(1)
    mode, nbytes, dropped = ix.screen_state()
    assert mode == 1 and nbytes > 5000 * 768 and not dropped
    monkeypatch.setenv("RFX_SCREEN_MAX_BYTES", str(nbytes))  # exactly the current copy: no room to grow
    first = ix.add_synthetic(3, 200_000, gen_row0=5000)  # grows the capacity: the copy cannot follow
    assert first == 5000 and ix.rows == 205_000
    assert ix.screen_state() == (0, 0, True) and ix.search_plan(256, 10) == 6
    exact = DeviceIndex(768, "bf16", 0)
    exact.add_synthetic(3, 205_000)
    q = synth_rows(4, 0, 256, 768, "bf16")
    a, b = ix.search(q, 10), exact.search(q, 10)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    monkeypatch.delenv("RFX_SCREEN_MAX_BYTES")
    ix.enable_screen(1)  # room again: the copy is rebuilt and the two-pass plan is back
    assert ix.screen_state()[0] == 1 and not ix.screen_state()[2] and ix.search_plan(256, 10) == 10
    a = ix.search(q, 10)  # one score rule for every plan (fl32 of the f64 dot): the two-pass
    # answer and the exact scan's re-scored answer carry the same bits
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])


def test_store_upload_past_the_cap_commits_and_answers_exactly(tmp_path, monkeypatch):
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_SCREEN", "1")
    monkeypatch.setenv("RFX_SCREEN_MAX_BYTES", "4096")
    ret = GpuRetriever(registry=rstore.StoreRegistry(root=str(tmp_path), device=0), dtype="bf16")
    name = ret.create_store("capped")
    fid, n = ret.add_document(name, "alpha beta gamma delta epsilon zeta " * 40, "doc0",
                              {"white_space_config": {"max_tokens_per_chunk": 4}}, None)
    assert fid.startswith("files/") and n > 0
    st = ret.registry.get(name)
    assert st._screen_on is None and st.index.screen_state()[0] == 0
    assert st.index.search_plan(256, 10) == 6 and st.index.search_plan(1, 10) == 0
    hits = ret.search([name], "alpha gamma", 5)
    assert len(hits) == 5 and all(h.file_id == fid for h in hits)
    other = GpuRetriever(registry=rstore.StoreRegistry(root=str(tmp_path), device=0), dtype="bf16")
    assert [(h.row, h.score) for h in other.search([name], "alpha gamma", 5)] == [(h.row, h.score) for h in hits]


WS4 = {"white_space_config": {"max_tokens_per_chunk": 4}}
QUESTIONS = ["alpha gamma", "theta kappa lambda", "document retrieval", "roofline lds", "beta zeta assistant"]


def _doc(i, words):
    vocab = ["alpha", "beta", "gamma", "delta", "theta", "kappa", "lambda", "document", "retrieval", "roofline",
             "lds", "zeta", "assistant", "citations", "wavefront", "matrix"]
    return " ".join(f"{vocab[(i * 7 + j * 5) % len(vocab)]}{(i * 31 + j) % 97}" if j % 3 else vocab[(i + j) % len(vocab)]
                    for j in range(words))


def test_sharded_store_drops_every_copy_when_the_last_shard_outgrows_it(tmp_path, monkeypatch):
    """only the last shard of a row-sharded store takes appends, so only it can outgrow
    its int8 copy.  The store must then answer with one plan: every shard drops its copy, the store
    records it (_screen_on None), and the answers equal an unsharded exact store bit for bit."""
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    root = str(tmp_path)
    monkeypatch.setenv("RFX_SCREEN", "1")
    writer = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
    name = writer.create_store("grow")
    writer.add_document(name, _doc(0, 24_000), "doc0", WS4, None)
    sharded = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0, devices="0x4"), dtype="bf16")
    st = sharded.registry.get(name)
    six = st.index
    assert st._screen_on is True and all(sh.screen_state()[0] == 1 for sh in six.shards)
    cap = max(sh.screen_state()[1] for sh in six.shards)
    monkeypatch.setenv("RFX_SCREEN_MAX_BYTES", str(cap))  # no shard's copy may grow from here
    writer.add_document(name, _doc(1, 40_000), "doc1", WS4, None)  # grows the last shard's capacity
    hits = {q: [(h.row, h.score) for h in sharded.search([name], q, 10)] for q in QUESTIONS}  # (catches up)
    st = sharded.registry.get(name)
    six = st.index
    assert st._screen_on is None
    mode, nbytes, dropped = six.screen_state()
    assert mode == 0 and nbytes == 0 and dropped
    assert all(sh.screen_state()[0] == 0 and sh.search_plan(256, 10) != 10 for sh in six.shards)
    monkeypatch.setenv("RFX_SCREEN", "0")
    monkeypatch.delenv("RFX_SCREEN_MAX_BYTES")
    plain = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
    pst = plain.registry.get(name)
    assert pst._screen_on is False and pst.index.search_plan(256, 10) != 10
    for q in QUESTIONS:
        assert hits[q] == [(h.row, h.score) for h in plain.search([name], q, 10)], q
    emb = plain.embedder(768)
    qs = emb.embed_texts([f"{w} {v}" for w in ("alpha", "theta", "roofline", "lds") for v in range(64)], "bf16")
    a_s, a_r = pst.index.search(qs, 10)
    b_s, b_r = six.search(qs, 10)
    assert torch.equal(a_r, b_r) and torch.equal(a_s, b_s)


def test_union_over_a_member_that_dropped_its_copy(tmp_path, monkeypatch):
    """A union view keeps an int8 copy only when every member does (each member's real state, not the
    first member's): after one member's copy is dropped by growth the view is rebuilt without one, and
    the union answers exactly as the per-store path does."""
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_SCREEN", "1")
    ret = GpuRetriever(registry=rstore.StoreRegistry(root=str(tmp_path), device=0), dtype="bf16")
    ret.batching = False
    names = [ret.create_store(f"u{i}") for i in range(2)]
    for i, nm in enumerate(names):
        ret.add_document(nm, _doc(10 + i, 6_000), f"doc{i}", WS4, None)
    sts = [ret.registry.get(nm) for nm in names]
    assert all(s._screen_on is True for s in sts)

    def both_paths():
        out = []
        for q in QUESTIONS:
            ret.union = True
            a = [(h.score, h.store, h.row) for h in ret.search(names, q, 10)]
            assert ret.last_path == "union"
            ret.union = False
            b = [(h.score, h.store, h.row) for h in ret.search(names, q, 10)]
            assert a == b, q
            out.append(a)
        return out

    both_paths()
    view = next(iter(ret._unions.values()))[0] if hasattr(ret, "_unions") else None
    cap = sts[1].index.screen_state()[1]
    monkeypatch.setenv("RFX_SCREEN_MAX_BYTES", str(cap))
    ret.add_document(names[1], _doc(20, 30_000), "grow", WS4, None)  # member 1 outgrows its copy
    assert ret.registry.get(names[1])._screen_on is None and ret.registry.get(names[0])._screen_on is True
    both_paths()
    from rfx import union as runion
    assert not runion.members_screened([ret.registry.get(nm) for nm in names])
    if view is not None:
        assert view.screened
