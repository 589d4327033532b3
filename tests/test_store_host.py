"""CPU: the append-only store protocol (rfx/store.py) with the host stand-in index (tests/fakes.py
HostIndex, same row-file format as rfx_rows_append / rfx_rows_sync).

Covers SURVEY §8f item 1 / VERDICT r1 item 8: uploads cost O(own rows); another process (API)
catches up incrementally; a crashed writer's torn tail is ignored and cut; two worker processes
appending to one store lose nothing; a busy writer lock maps to TimeoutError (retryable,
gemini_rag.py:17-27); a store dropped by another process disappears from every registry."""
import fcntl
import json
import multiprocessing as mp
import os

import numpy as np
import pytest

from fakes import HostIndex
from rfx import store as rstore


def reg(root):
    return rstore.StoreRegistry(root=str(root), device=0, index_factory=HostIndex)


def vecs(n, seed, dim=64):
    return np.random.default_rng(seed).standard_normal((n, dim)).astype(np.float32)


def test_roundtrip_other_process_view(tmp_path):
    a = reg(tmp_path)
    st = a.create("demo", 64, "f32")
    f1, first1 = st.add_document(["c0", "c1", "c2"], vecs(3, 1), "one.md", {"tenant": "acme"})
    f2, first2 = st.add_document(["d0"], vecs(1, 2), "two.md")
    assert (first1, first2) == (0, 3)
    b = reg(tmp_path)  # another process: opens from disk
    sb = b.get(st.name)
    assert sb.rows == st.rows and sb.index.rows == 4
    assert np.array_equal(sb.index.data, st.index.data)
    assert sb.files[f1]["metadata"] == {"tenant": "acme"} and sb.files[f2]["first"] == 3
    assert sb.row_info(3)[:3] == (f2, "d0", "two.md") and sb.row_info(4) is None


def test_incremental_catch_up(tmp_path):
    a, b = reg(tmp_path), reg(tmp_path)
    st = a.create("demo", 64, "f32")
    st.add_document(["x"] * 5, vecs(5, 1), "a")
    sb = b.get(st.name)
    assert sb.index.rows == 5
    HostIndex.syncs.clear()
    st.add_document(["y"] * 2, vecs(2, 2), "b")
    fid = st.add_document(["z"] * 3, vecs(3, 3), "c")[0]
    st.delete_file(fid)
    sb2 = b.get(st.name)
    assert sb2 is sb  # same object, caught up in place
    assert [s[1:] for s in HostIndex.syncs] == [(5, 10)]  # only the appended rows were read
    assert sb.index.rows == 10 and len(sb.rows) == 10
    assert sb.files[fid]["deleted"] and np.isnan(sb.index.data[7:10]).all()
    assert not np.isnan(sb.index.data[:7]).any()


def test_writer_catches_up_before_appending(tmp_path):
    a, b = reg(tmp_path), reg(tmp_path)
    st = a.create("demo", 64, "f32")
    sb = b.get(st.name)
    st.add_document(["a"] * 4, vecs(4, 1), "a")
    _, first = sb.add_document(["b"] * 2, vecs(2, 2), "b")  # b never saw a's rows before
    assert first == 4
    c = reg(tmp_path).get(st.name)
    assert c.index.rows == 6 and [r[1] for r in c.rows] == ["a"] * 4 + ["b"] * 2


def test_torn_tail_is_ignored_and_cut(tmp_path):
    a = reg(tmp_path)
    st = a.create("demo", 64, "f32")
    st.add_document(["a"] * 2, vecs(2, 1), "a")
    # a writer died after appending rows + metadata but before its manifest commit
    with open(os.path.join(st.path, "rows.rfx"), "ab") as f:
        f.write(b"\x7f" * 64 * 4 * 3 + b"\x01\x02")
    with open(os.path.join(st.path, "meta.jsonl"), "ab") as f:
        f.write(b'{"f": "files/local-dead", "t": "half')
    b = reg(tmp_path).get(st.name)
    assert b.index.rows == 2 and len(b.rows) == 2
    st.add_document(["c"], vecs(1, 3), "c")
    c = reg(tmp_path).get(st.name)
    assert c.index.rows == 3 and [r[1] for r in c.rows] == ["a", "a", "c"]
    assert os.path.getsize(os.path.join(st.path, "rows.rfx")) == 64 + 3 * 64 * 4


def test_dropped_by_another_process(tmp_path):
    a, b = reg(tmp_path), reg(tmp_path)
    st = a.create("demo", 64, "f32")
    st.add_document(["a"], vecs(1, 1), "a")
    sb = b.get(st.name)
    evicted = []
    b.on_evict.append(evicted.append)
    assert a.drop(st.name)
    assert b.get(st.name) is None and evicted == [st.name] and sb.index.closed
    assert st.name not in b.names()


def test_writer_lock_timeout_is_retryable(tmp_path, monkeypatch):
    a = reg(tmp_path)
    st = a.create("demo", 64, "f32")
    monkeypatch.setenv("RFX_LOCK_TIMEOUT_S", "0.2")
    fd = os.open(os.path.join(st.path, ".lock"), os.O_RDWR)
    fcntl.flock(fd, fcntl.LOCK_EX)  # another writer holds the store
    try:
        with pytest.raises(TimeoutError):
            st.add_document(["a"], vecs(1, 1), "a")
    finally:
        fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)
    st.add_document(["a"], vecs(1, 1), "a")
    assert reg(tmp_path).get(st.name).index.rows == 1


def _writer(root, name, tag, n_docs, q):
    try:
        r = reg(root)
        st = r.get(name)
        for i in range(n_docs):
            st.add_document([f"{tag}{i}-{j}" for j in range(i % 3 + 1)], vecs(i % 3 + 1, hash((tag, i)) % 1000),
                            f"{tag}{i}")
        q.put(None)
    except BaseException as e:  # report to the parent
        q.put(repr(e))


def test_two_processes_append_concurrently(tmp_path):
    st = reg(tmp_path).create("demo", 64, "f32")
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_writer, args=(str(tmp_path), st.name, tag, 25, q)) for tag in "AB"]
    for p in ps:
        p.start()
    errs = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert errs == [None, None]
    fin = reg(tmp_path).get(st.name)
    n = sum(i % 3 + 1 for i in range(25)) * 2
    assert fin.index.rows == n and len(fin.rows) == n
    # every file's rows are contiguous, disjoint, and carry that file's chunk texts
    spans = sorted((f["first"], f["n"], f["display_name"]) for f in fin.files.values())
    pos = 0
    for first, cnt, title in spans:
        assert first == pos
        assert all(fin.rows[first + j][1] == f"{title}-{j}" for j in range(cnt))
        pos += cnt
    assert pos == n
    man = json.load(open(os.path.join(st.path, "manifest.json")))
    assert man["version"] == 50 and man["rows"] == n


@pytest.mark.parametrize("op", ["add", "delete"])
def test_failed_file_record_append_rolls_back(tmp_path, monkeypatch, op):
    """a failure in the files.jsonl append (after the rows and metadata were written)
    must leave this writer in the committed state: no phantom rows, and the next upload commits
    a consistent store that other processes can open."""
    a = reg(tmp_path)
    st = a.create("demo", 64, "f32")
    fid, _ = st.add_document(["c0", "c1"], vecs(2, 1), "one.md")
    real = rstore._append

    def failing(path, committed, data):
        if path.endswith("files.jsonl"):
            raise OSError(28, "No space left on device")
        return real(path, committed, data)

    monkeypatch.setattr(rstore, "_append", failing)
    with pytest.raises(OSError):
        if op == "add":
            st.add_document(["d0", "d1", "d2"], vecs(3, 2), "two.md")
        else:
            st.delete_file(fid)
    monkeypatch.setattr(rstore, "_append", real)
    assert st.index.rows == 2 and len(st.rows) == 2
    assert not st.files[fid]["deleted"] and not np.isnan(st.index.data).any()
    f3, first3 = st.add_document(["e0"], vecs(1, 3), "three.md")
    assert first3 == 2
    sb = reg(tmp_path).get(st.name)  # another process opens it without a row/metadata mismatch
    assert sb.index.rows == 3 and len(sb.rows) == 3 and sb.row_info(2)[0] == f3


class _NoRoomIndex(HostIndex):
    """A host index whose int8 copy never fits (librfx's RFX_ECAPACITY)."""
    calls = 0

    def enable_screen(self, mode=1):
        from rfx._lib import RfxCapacityError
        type(self).calls += 1
        raise RfxCapacityError(7, "int8 copy of 3 rows needs 2304 B > RFX_SCREEN_MAX_BYTES 0 (test)")


def test_screen_capacity_never_fails_a_committed_upload(tmp_path, monkeypatch):
    """VERDICT r3 missing #2: the copy is built after the manifest commit; when it does not fit, the
    upload still returns its file id (no ERROR document, ingestion.py:311-339), readers catch up without
    raising, and the store does not retry the copy on every upload of the same generation."""
    monkeypatch.setenv("RFX_SCREEN", "1")
    _NoRoomIndex.calls = 0
    w = rstore.StoreRegistry(root=str(tmp_path), device=0, index_factory=_NoRoomIndex)
    st = w.create("big", 768, "f32")
    f1, first1 = st.add_document(["a", "b"], vecs(2, 1, 768), "one.md")
    f2, first2 = st.add_document(["c"], vecs(1, 2, 768), "two.md")
    assert (first1, first2) == (0, 2) and st.index.rows == 3 and len(st.rows) == 3
    assert _NoRoomIndex.calls == 1 and st._screen_on is None
    r = rstore.StoreRegistry(root=str(tmp_path), device=0, index_factory=_NoRoomIndex).get(st.name)
    assert r.index.rows == 3 and r.files[f2]["first"] == 2
