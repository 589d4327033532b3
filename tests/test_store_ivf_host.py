"""CPU: the IVF store protocol (rfx/store.py, config 5 served from the store) with host stand-ins
for the device index and the IVF index (tests/fakes.py HostIndex, HostIvf).

Checks: no lists before train_min live rows; the writer trains once, on live rows only, and commits
the centroid file with the manifest; every other process loads exactly those centroids and grows
its lists by the appended rows only; deleted rows never come back from the re-rank; an 8x growth
retrains under a new centroid id that readers switch to; with nprobe = nlist the IVF answer is the
exact top-k; a filtered search and a flat store keep the exact scan."""
import json
import os

import numpy as np
import pytest

from fakes import HostIndex, HostIvf
from rfx import store as rstore

SPEC = {"kind": "ivf", "nlist": 4, "nprobe": 4, "train_min": 16}


def reg(root):
    return rstore.StoreRegistry(root=str(root), device=0, index_factory=HostIndex, ivf_factory=HostIvf)


def vecs(n, seed, dim=32):
    return np.random.default_rng(seed).standard_normal((n, dim)).astype(np.float32)


def exact(st, q, k):
    x = st.index.read(0, st.index.rows)
    out = []
    for qi in q:
        sc = x @ qi
        ok = np.flatnonzero(~np.isnan(sc))
        out.append(list(ok[np.lexsort((ok, -sc[ok]))][:k]))
    return out


def test_train_commit_and_reader_load(tmp_path):
    HostIvf.log.clear()
    a = reg(tmp_path)
    st = a.create("demo", 32, "f32", spec=SPEC)
    st.add_document(["a"] * 10, vecs(10, 1), "a.md")
    assert st.ivf is None and json.load(open(os.path.join(st.path, "manifest.json")))["ivf"] is None
    dead = st.add_document(["b"] * 4, vecs(4, 2), "b.md")[0]
    st.delete_file(dead)
    st.add_document(["c"] * 8, vecs(8, 3), "c.md")  # 18 live rows >= train_min
    man = json.load(open(os.path.join(st.path, "manifest.json")))
    assert man["index"] == SPEC and man["ivf"]["rows"] == 18
    assert ("train", 18) in HostIvf.log  # the 4 deleted rows are not in the sample
    raw = open(os.path.join(st.path, f"ivf-{man['ivf']['id']}.bin"), "rb").read()
    assert raw[:8] == b"RFXCENT1" and len(raw) == 20 + 4 * 32
    assert raw[20:] == st.ivf.centroid_bytes() and st.ivf_ready()

    b = reg(tmp_path)  # another process
    sb = b.get(st.name)
    assert sb.ivf_ready() and sb.ivf.centroid_bytes() == raw[20:]
    assert np.array_equal(sb.ivf.labels, st.ivf.labels)
    q = vecs(5, 9)
    for s in (st, sb):
        got_s, got_r = s.search(q, 6)
        assert [list(r) for r in got_r.numpy()] == exact(s, q, 6)  # nprobe = nlist: exact
        assert not np.isin(got_r.numpy(), np.arange(10, 14)).any()


def test_reader_grows_lists_incrementally_and_switches_on_retrain(tmp_path):
    a, b = reg(tmp_path), reg(tmp_path)
    st = a.create("demo", 32, "f32", spec=SPEC)
    st.add_document(["a"] * 20, vecs(20, 1), "a.md")
    sb = b.get(st.name)
    cid = sb.ivf_id
    HostIvf.log.clear()
    st.add_document(["b"] * 7, vecs(7, 2), "b.md")
    assert b.get(st.name) is sb and sb.ivf_id == cid
    assert [e for e in HostIvf.log if e[0] == "add"] == [("add", 20, 27), ("add", 20, 27)]  # writer + reader
    st.add_document(["c"] * 140, vecs(140, 3), "c.md")  # 167 >= 8 x 20: retrain
    b.get(st.name)
    assert st.ivf_id != cid and sb.ivf_id == st.ivf_id and sb.ivf.rows == 167
    assert st.ivf_meta == {"id": st.ivf_id, "rows": 167}
    assert os.path.exists(os.path.join(st.path, f"ivf-{cid}.bin"))  # old centroids stay readable


def test_filtered_and_flat_searches_use_the_exact_scan(tmp_path, monkeypatch):
    calls = []
    monkeypatch.setattr(HostIndex, "search", lambda self, q, k, row_mask=None: calls.append(row_mask) or "scan",
                        raising=False)
    a = reg(tmp_path)
    st = a.create("demo", 32, "f32", spec=SPEC)
    st.add_document(["a"] * 20, vecs(20, 1), "a.md")
    assert st.search(vecs(1, 5), 3, row_mask="mask") == "scan" and calls == ["mask"]
    flat = a.create("flat", 32, "f32", spec={"kind": "flat"})
    flat.add_document(["a"] * 40, vecs(40, 1), "a.md")
    assert flat.ivf is None and flat.search(vecs(1, 5), 3) == "scan"


def test_env_spec(monkeypatch):
    monkeypatch.setenv("RFX_INDEX", "ivf")
    monkeypatch.setenv("RFX_IVF_NLIST", "256")
    assert rstore.index_spec_from_env() == {"kind": "ivf", "nlist": 256, "nprobe": 32, "train_min": 8192}
    monkeypatch.setenv("RFX_INDEX", "hnsw")
    with pytest.raises(ValueError):
        rstore.index_spec_from_env()
    monkeypatch.delenv("RFX_INDEX")
    assert rstore.index_spec_from_env() == {"kind": "flat"}


def test_corrupt_centroid_file_fails_loudly(tmp_path):
    a = reg(tmp_path)
    st = a.create("demo", 32, "f32", spec=SPEC)
    st.add_document(["a"] * 20, vecs(20, 1), "a.md")
    p = os.path.join(st.path, f"ivf-{st.ivf_id}.bin")
    open(p, "r+b").truncate(30)
    with pytest.raises(RuntimeError, match="malformed"):
        reg(tmp_path).get(st.name)
