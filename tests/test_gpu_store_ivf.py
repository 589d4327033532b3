"""GPU: an IVF store (SURVEY §8 config 5 served from the store, rfx/store.py) on the HIP path.

The writer trains when the live rows reach train_min: the committed centroid file is BIT-EXACT
with oracle/ivf.py's k-means over the same sample (the live rows, strided), so every process
holds the oracle's quantiser.  Unfiltered searches go through the lists and the exact re-rank
against the DeviceIndex rows: scores within 1e-5 of the oracle's f64 dot of the stored row,
tombstoned rows never returned, recall@10 against the exact scan >= 0.9 at nprobe 8 of 32 on
clustered rows, and a second registry (another process's view) answers bit-identically."""
import os

import numpy as np
import pytest
import torch

from oracle import ivf as oivf

pytestmark = pytest.mark.gpu

DIM, NLIST = 768, 32
SPEC = {"kind": "ivf", "nlist": NLIST, "nprobe": 8, "train_min": 4000}


def to_np_bf16(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def test_ivf_store_train_search_reader(tmp_path):
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    from rfx import ivf as rivf
    from rfx import store as rstore
    from rfx.quality import recall_at_k

    reg = rstore.StoreRegistry(root=str(tmp_path), device=0)
    st = reg.create("ivf-demo", DIM, "bf16", spec=SPEC)
    docs = [rivf.synth_clustered(7, 48, 100 + i, 1500 * i, 1500, DIM, "bf16") for i in range(4)]
    fids = []
    for i, v in enumerate(docs[:3]):
        fids.append(st.add_document([f"d{i}-{j}" for j in range(1500)], v, f"d{i}.md", {"tenant": f"t{i}"})[0])
        if i == 1:
            st.delete_file(fids[1])
    assert st.ivf is None  # 3000 live rows < train_min
    st.add_document([f"d3-{j}" for j in range(1500)], docs[3], "d3.md")
    assert st.ivf_ready() and st.ivf_meta["rows"] == 4500

    # centroids: bit-exact with the oracle's k-means over the same sample
    all_rows = np.concatenate([to_np_bf16(v) for v in docs])
    live = np.concatenate([np.arange(0, 1500), np.arange(3000, 6000)])
    sample = live[::max(1, live.size // (64 * NLIST))]
    sq, _ = oivf.quantize(oivf.stored_to_f32(all_rows[sample], "bf16"))
    qc, _ = oivf.train(sq, NLIST, 10)
    raw = open(os.path.join(st.path, f"ivf-{st.ivf_id}.bin"), "rb").read()
    assert np.array_equal(np.frombuffer(raw[20:], dtype=np.int8).reshape(NLIST, DIM), qc)

    q = rivf.synth_clustered(7, 48, 999, 0, 40, DIM, "bf16")
    s, r = st.search(q, 10)
    es, er = st.index.search(q, 10)
    s, r, es, er = s.numpy(), r.numpy(), es.cpu().numpy(), er.cpu().numpy()
    assert not np.isin(r, np.arange(1500, 3000)).any(), "a deleted row came back"
    assert recall_at_k(r.tolist(), er.tolist(), 10) >= 0.9
    rows64 = oivf.stored_to_f32(all_rows, "bf16").astype(np.float64)
    q64 = oivf.stored_to_f32(to_np_bf16(q), "bf16").astype(np.float64)
    for i in range(len(q)):
        ok = r[i] >= 0
        assert np.all(np.abs(s[i][ok] - rows64[r[i][ok]] @ q64[i]) <= 1e-5)
        assert np.all(np.diff(s[i][ok]) <= 0)

    # another process's view: same centroids, same lists, bit-identical answers
    other = rstore.StoreRegistry(root=str(tmp_path), device=0).get(st.name)
    assert other.ivf_ready() and other.ivf_id == st.ivf_id
    s2, r2 = other.search(q, 10)
    assert np.array_equal(r2.numpy(), r) and np.array_equal(s2.numpy().view(np.uint32), s.view(np.uint32))

    # a filtered search (row mask) keeps the exact scan
    mask = st.row_mask({"tenant": "t0"})
    fs, fr = st.search(q, 10, row_mask=mask)
    xs, xr = st.index.search(q, 10, row_mask=mask)
    assert torch.equal(fr, xr) and torch.equal(fs, xs) and int(fr.max()) < 1500
    other.close()
    reg.drop(st.name)


def test_ivf_store_behind_retriever(tmp_path, monkeypatch):
    """GpuRetriever over an RFX_INDEX=ivf store returns the same hits as over a flat store when
    every list is probed (nprobe = nlist, re-rank depth 2k >= the candidates that matter)."""
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_INDEX", "ivf")
    monkeypatch.setenv("RFX_IVF_NLIST", "4")
    monkeypatch.setenv("RFX_IVF_NPROBE", "4")
    monkeypatch.setenv("RFX_IVF_TRAIN_MIN", "8")
    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path / "ivf"), device=0))
    ret = GpuRetriever(dtype="bf16")
    text = " ".join(f"word{i % 97} topic{i % 13}" for i in range(3000))
    si = ret.create_store("ivf")
    ret.add_document(si, text, "t.md", {"white_space_config": {"max_tokens_per_chunk": 16, "max_overlap_tokens": 2}})
    assert rstore.registry().get(si).ivf_ready()
    monkeypatch.setenv("RFX_INDEX", "flat")
    sf = ret.create_store("flat")
    ret.add_document(sf, text, "t.md", {"white_space_config": {"max_tokens_per_chunk": 16, "max_overlap_tokens": 2}})
    for qtext in ["word5 topic3", "topic12 word96 word1", "word40 word41 topic0"]:
        a = {h.row: h.score for h in ret.search([si], qtext, 5)}
        b = ret.search([sf], qtext, 6)
        exact = {h.row: h.score for h in b[:5]}
        if b[4].score - b[5].score > 1e-4:  # no near-tie at the cut: the same five rows
            assert set(a) == set(exact)
        for row in set(a) & set(exact):
            assert abs(a[row] - exact[row]) <= 1e-5
