"""GPU: the append-only store (rfx/store.py) on the real HIP index (rfx_rows_append / rfx_rows_sync):
two worker processes append to one store at once, another process catches up incrementally, and
every stored vector is bit-identical to the embedding of its chunk (nothing lost or torn)."""
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(root, name, tag, n_docs, q):
    try:
        from rfx import store as rstore
        from rfx.retriever import GpuRetriever

        torch.cuda.set_device(0)
        rstore.set_registry(rstore.StoreRegistry(root=root, device=0))
        ret = GpuRetriever(dtype="bf16")
        for i in range(n_docs):
            words = " ".join(f"{tag}{i}w{j}" for j in range(7 + i % 5))
            ret.add_document(name, words, f"{tag}-{i}", {"white_space_config": {"max_tokens_per_chunk": 3,
                                                                                 "max_overlap_tokens": 1}})
        q.put(None)
    except BaseException as e:
        q.put(repr(e))


def _bits(t):
    return t.cpu().view(torch.int16).numpy()


def test_two_writer_processes_and_incremental_reader(tmp_path):
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    root = str(tmp_path)
    rstore.set_registry(rstore.StoreRegistry(root=root, device=0))
    ret = GpuRetriever(dtype="bf16")
    name = ret.create_store("shared")
    st = rstore.registry().get(name)
    assert st.index.rows == 0

    ctx = mp.get_context("spawn")  # fresh HIP state per child
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(root, name, tag, 12, q)) for tag in "AB"]
    for p in ps:
        p.start()
    errs = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert errs == [None, None]

    st2 = rstore.registry().get(name)  # this process catches up in place
    assert st2 is st
    n = st.index.rows
    assert n == len(st.rows) and n > 0 and len(st.files) == 24
    # every file's rows are contiguous and hold exactly the embeddings of its chunks
    emb = ret.embedder(768)
    pos = 0
    for f in sorted(st.files.values(), key=lambda f: f["first"]):
        assert f["first"] == pos
        texts = [st.rows[f["first"] + j][1] for j in range(f["n"])]
        want = emb.embed_texts(texts, "bf16")
        got = st.index.read(f["first"], f["n"])
        assert np.array_equal(_bits(got), _bits(want)), f["display_name"]
        pos += f["n"]
    assert pos == n
    # a fresh process view (full open) equals the incrementally synced one, and retrieval works
    other = rstore.StoreRegistry(root=root, device=0).get(name)
    assert np.array_equal(_bits(other.index.read(0, n)), _bits(st.index.read(0, n)))
    hits = ret.search([name], "A3w1 A3w2", 3)
    assert hits and hits[0].title == "A-3"


def test_delete_visible_to_other_process_view(tmp_path):
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    root = str(tmp_path)
    rstore.set_registry(rstore.StoreRegistry(root=root, device=0))
    ret = GpuRetriever(dtype="f32")
    name = ret.create_store("s")
    fa, _ = ret.add_document(name, "alpha beta gamma delta", "a", {"white_space_config": {"max_tokens_per_chunk": 2,
                                                                                          "max_overlap_tokens": 0}})
    ret.add_document(name, "epsilon zeta eta theta", "b", {"white_space_config": {"max_tokens_per_chunk": 2,
                                                                                  "max_overlap_tokens": 0}})
    other = rstore.StoreRegistry(root=root, device=0)
    assert other.get(name).index.live_rows == 4
    assert ret.delete_file(name, fa)
    ost = other.get(name)
    assert ost.index.live_rows == 2 and ost.files[fa]["deleted"]
    assert os.path.getsize(os.path.join(ost.path, "tombs.bin")) == 16
