"""Local File-Search-store equivalent: a DeviceIndex plus per-row chunk metadata, persisted on
disk so that the API processes serve what the ingestion worker wrote (the worker deletes the
uploaded file after indexing, backend/app/services/ingestion.py:341) — SURVEY §8f item 1.

On-disk layout of a store (directory <root>/<store id>/), every data file APPEND-ONLY:
  rows.rfx      rfx_rows_append() row file: 64-byte header + row-major rows (C ABI, include/rfx.h)
  meta.jsonl    one JSON object per row: {"f": file_id, "t": chunk text}
  files.jsonl   file records: {"op": "add", "id", "first", "n", "display_name", "uri", "metadata"}
                and {"op": "del", "id"}
  tombs.bin     int64 row ids of deleted rows
  ivf-<id>.bin  (IVF stores) k-means centroids: "RFXCENT1", u32 nlist, u32 dim, 4 zero bytes,
                then int8 [nlist][dim]; written once per training, never modified
  manifest.json the commit point: {"format": 2, "name", "display_name", "dim", "dtype",
                "generation", "version", "rows", "meta_bytes", "files_bytes", "tombs",
                "index": {"kind": "flat"|"ivf", "nlist", "nprobe", "train_min"},
                "ivf": null | {"id", "rows"}} — the committed length of every file above;
                replaced atomically (rename) after the appended bytes are fsync'ed.  Readers
                never read past it, so a writer that dies mid-append leaves a tail that is
                ignored, and cut by the next writer.
  .lock         fcntl writer lock: appends from several processes (ARQ worker max_jobs=10,
                worker.py:125; several workers) serialise on it, each first catching up with
                what the others committed.
An upload costs O(its own rows) of disk and device work; a reader (API process) that sees a
newer manifest loads only what was appended since its last look (rows, metadata, tombstones).

IVF stores (RFX_INDEX=ivf at creation): the writer trains k-means on the
live rows once there are train_min of them (again at every 8x growth) and commits the centroids
file with the manifest; every process keeps an IvfIndex (rfx.ivf) over the same rows in the same
order, built from the committed centroids and extended incrementally as rows arrive.  Unfiltered
searches probe nprobe lists and re-rank the candidates exactly against the DeviceIndex rows (so
tombstones, NaN there, never return); filtered searches and untrained stores use the exact scan.

GPU state is a process-level singleton (StoreRegistry), because get_rag_client() builds a new
adapter per request (chat.py:937, ingestion.py:214).
"""
import errno
import fcntl
import json
import logging
import os
import shutil
import threading
import time
import uuid

import numpy as np

from . import filters
from ._lib import RFX_EBUSY, RfxError, RfxTransientError
from .index import DeviceIndex

log = logging.getLogger("rfx.store")

STORE_PREFIX = "fileSearchStores/"  # accepted by routes/stores.py:46 (prefix check)
FORMAT = 2
_CENT_MAGIC = b"RFXCENT1"


def index_spec_from_env():
    """Index kind of new stores: RFX_INDEX=flat (default, exact scan) | ivf (RFX_IVF_NLIST lists,
    default 1024; RFX_IVF_NPROBE, default 32; trained at RFX_IVF_TRAIN_MIN live rows, default
    32 x nlist)."""
    kind = os.environ.get("RFX_INDEX", "flat")
    if kind == "flat":
        return {"kind": "flat"}
    if kind != "ivf":
        raise ValueError(f"RFX_INDEX={kind!r}: expected flat or ivf")
    nlist = int(os.environ.get("RFX_IVF_NLIST", "1024"))
    return {"kind": "ivf", "nlist": nlist, "nprobe": min(int(os.environ.get("RFX_IVF_NPROBE", "32")), nlist, 64),
            "train_min": int(os.environ.get("RFX_IVF_TRAIN_MIN", str(32 * nlist)))}


def default_root() -> str:
    return os.environ.get("RFX_INDEX_DIR", os.path.join(os.path.expanduser("~"), ".cache", "rfx", "stores"))


def _fsync_dir(path):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _append(path, committed, data: bytes) -> int:
    """Cut `path` to its committed length (drops a crashed writer's tail), append data, fsync.
    Returns the new committed length."""
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_CLOEXEC, 0o644)
    try:
        os.ftruncate(fd, committed)
        os.lseek(fd, committed, os.SEEK_SET)
        view = memoryview(data)
        while view:
            n = os.write(fd, view)
            view = view[n:]
        os.fsync(fd)
    finally:
        os.close(fd)
    return committed + len(data)


def _read_range(path, start, end) -> bytes:
    if end <= start:
        return b""
    with open(path, "rb") as f:
        f.seek(start)
        b = f.read(end - start)
    if len(b) != end - start:
        raise OSError(errno.EIO, f"{path}: committed range [{start}, {end}) is missing")
    return b


class StoreGone(Exception):
    """The store's manifest no longer exists (dropped by another process)."""


class LocalStore:
    # the vector store behind a LocalStore: DeviceIndex (HIP) in the product; tests inject a host
    # stand-in with the same interface to exercise the file protocol without a GPU
    index_factory = DeviceIndex
    ivf_factory = None  # rfx.ivf.IvfIndex (imported on first use); tests inject a host stand-in

    def __init__(self, path, device, index_factory=None, ivf_factory=None):
        self.path, self.device = path, int(device)
        if index_factory is not None:
            self.index_factory = index_factory
        if ivf_factory is not None:
            self.ivf_factory = ivf_factory
        self.name = self.display_name = None
        self.dim = self.dtype = None
        self.generation = None
        self.index = None
        self.rows = []      # per row: (file_id, chunk text)
        self.files = {}     # file_id -> {"first", "n", "display_name", "uri", "deleted", "metadata"}
        self.version = -1
        self.meta_bytes = self.files_bytes = self.tombs = 0
        self.lock = threading.RLock()
        self._stat = None
        self._masks = {}    # (version, filter key) -> device row mask
        self._screen_on = False  # the index holds the two-pass scan's int8 copy (_maybe_screen)
        self.spec = {"kind": "flat"}
        self.ivf_meta = None  # committed {"id", "rows"} of the current centroids
        self.ivf = None       # this process's IvfIndex over the committed rows
        self.ivf_id = None

    # ---- files -------------------------------------------------------------------------------
    def _p(self, name):
        return os.path.join(self.path, name)

    def _read_manifest(self):
        try:
            with open(self._p("manifest.json"), encoding="utf-8") as f:
                st = os.fstat(f.fileno())
                man = json.load(f)
        except FileNotFoundError:
            return None, None
        if man.get("format") != FORMAT:
            raise RuntimeError(f"{self.path}: store format {man.get('format')} != {FORMAT}")
        return man, (st.st_ino, st.st_mtime_ns, st.st_size)

    def _write_manifest(self):
        man = {"format": FORMAT, "name": self.name, "display_name": self.display_name, "dim": self.dim,
               "dtype": self.dtype, "generation": self.generation, "version": self.version,
               "rows": len(self.rows), "meta_bytes": self.meta_bytes, "files_bytes": self.files_bytes,
               "tombs": self.tombs, "index": self.spec, "ivf": self.ivf_meta}
        tmp = self._p(f"manifest.json.{os.getpid()}.{threading.get_ident()}.tmp")
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(man, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self._p("manifest.json"))
        _fsync_dir(self.path)
        st = os.stat(self._p("manifest.json"))
        self._stat = (st.st_ino, st.st_mtime_ns, st.st_size)

    class _WriterLock:
        """fcntl lock on <store>/.lock, bounded wait -> RfxTransientError (a TimeoutError: the
        ingestion retry, ingestion.py:35-52, and RETRYABLE_EXCEPTIONS, gemini_rag.py:17-27)."""

        def __init__(self, store):
            self.path = store._p(".lock")
            self.timeout = float(os.environ.get("RFX_LOCK_TIMEOUT_S", "30"))

        def __enter__(self):
            try:
                self.fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_CLOEXEC, 0o644)
            except FileNotFoundError:
                raise StoreGone(self.path)
            t_end = time.monotonic() + self.timeout
            while True:
                try:
                    fcntl.flock(self.fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
                    return self
                except BlockingIOError:
                    if time.monotonic() >= t_end:
                        os.close(self.fd)
                        raise RfxTransientError(RFX_EBUSY, f"store writer lock {self.path} busy "
                                                           f"for {self.timeout:.0f} s")
                    time.sleep(0.005)

        def __exit__(self, *exc):
            fcntl.flock(self.fd, fcntl.LOCK_UN)
            os.close(self.fd)

    # ---- create / open / catch up ---------------------------------------------------------------
    @classmethod
    def create(cls, path, name, display_name, dim, dtype, device, index_factory=None, spec=None,
               ivf_factory=None):
        os.makedirs(path, exist_ok=False)
        st = cls(path, device, index_factory, ivf_factory)
        st.name, st.display_name, st.dim, st.dtype = name, display_name, int(dim), dtype
        st.spec = dict(spec or {"kind": "flat"})
        st.generation = uuid.uuid4().hex
        st.index = st.index_factory(st.dim, dtype, st.device)
        st.version = 0
        with st._WriterLock(st):
            st._write_manifest()
        return st

    @classmethod
    def open(cls, path, device, index_factory=None, ivf_factory=None):
        st = cls(path, device, index_factory, ivf_factory)
        with st.lock:
            st._sync()
        return st

    def _reset(self, man):
        self.name, self.display_name = man["name"], man["display_name"]
        self.dim, self.dtype = int(man["dim"]), man["dtype"]
        self.generation = man["generation"]
        if self.index is not None:
            self.index.close()
        self.index = self.index_factory(self.dim, self.dtype, self.device)
        self.spec = man.get("index") or {"kind": "flat"}
        self.ivf_meta = None
        self._drop_ivf()
        self.rows, self.files = [], {}
        self.meta_bytes = self.files_bytes = self.tombs = 0
        self.version = -1
        self._masks = {}
        self._screen_on = False

    def _sync(self, man=None, stat=None):
        """Catch up with the committed state on disk (caller holds self.lock).  Incremental: only
        what was appended since the last sync is read."""
        if man is None:
            man, stat = self._read_manifest()
        if man is None:
            raise StoreGone(self.path)
        if man["generation"] != self.generation:
            self._reset(man)
        if man["version"] == self.version:
            self._stat = stat
            return
        self.ivf_meta = man.get("ivf")
        n_rows = int(man["rows"])
        if n_rows < len(self.rows) or man["meta_bytes"] < self.meta_bytes or man["files_bytes"] < self.files_bytes \
                or man["tombs"] < self.tombs:
            raise RuntimeError(f"{self.path}: committed state went backwards (same generation)")
        if n_rows > self.index.rows:
            self.index.rows_sync(self._p("rows.rfx"), n_rows)
        for line in _read_range(self._p("meta.jsonl"), self.meta_bytes, man["meta_bytes"]).splitlines():
            o = json.loads(line)
            self.rows.append((o["f"], o["t"]))
        for line in _read_range(self._p("files.jsonl"), self.files_bytes, man["files_bytes"]).splitlines():
            self._apply_file_record(json.loads(line))
        if man["tombs"] > self.tombs:
            raw = _read_range(self._p("tombs.bin"), 8 * self.tombs, 8 * man["tombs"])
            self.index.tombstone(np.frombuffer(raw, dtype="<i8"))
        if len(self.rows) != n_rows or self.index.rows != n_rows:
            raise RuntimeError(f"{self.path}: {len(self.rows)} metadata rows / {self.index.rows} vectors, "
                               f"manifest says {n_rows}")
        self.meta_bytes, self.files_bytes, self.tombs = man["meta_bytes"], man["files_bytes"], man["tombs"]
        self.version = man["version"]
        self._stat = stat
        self._ivf_catch_up()
        self._maybe_screen()

    def _apply_file_record(self, r):
        if r["op"] == "add":
            self.files[r["id"]] = {"first": r["first"], "n": r["n"], "display_name": r["display_name"],
                                   "uri": r["uri"], "deleted": False, "metadata": r.get("metadata")}
        elif r["op"] == "del" and r["id"] in self.files:
            self.files[r["id"]]["deleted"] = True

    def stale(self) -> bool:
        """True when the manifest changed (or vanished) since this process last synced."""
        try:
            st = os.stat(self._p("manifest.json"))
        except FileNotFoundError:
            return True
        return (st.st_ino, st.st_mtime_ns, st.st_size) != self._stat

    def refresh(self) -> bool:
        """Catch up if another process committed; False when the store is gone."""
        with self.lock:
            try:
                self._sync()
            except StoreGone:
                return False
            return True

    # ---- writes (exclusive across processes) ------------------------------------------------------
    def add_document(self, chunks, vecs, display_name, metadata=None):
        with self.lock, self._WriterLock(self):
            self._sync()  # append at the end of what every writer committed
            file_id = f"files/local-{uuid.uuid4().hex}"
            first = self.index.rows
            # everything after the catch-up is one commit: any failure (ENOSPC, EIO, interrupt) in
            # the row, metadata, file-record or manifest writes re-reads the committed state, so no
            # phantom rows stay in this process's index
            try:
                if len(chunks):
                    self.index.add(vecs)
                    self.index.rows_append(self._p("rows.rfx"), first)
                    meta = "".join(json.dumps({"f": file_id, "t": c}, ensure_ascii=False) + "\n" for c in chunks)
                    self.meta_bytes = _append(self._p("meta.jsonl"), self.meta_bytes, meta.encode())
                rec = {"op": "add", "id": file_id, "first": first, "n": len(chunks), "display_name": display_name,
                       "uri": f"local://{self.name}/{file_id}", "metadata": metadata or None}
                self.files_bytes = _append(self._p("files.jsonl"), self.files_bytes, (json.dumps(rec) + "\n").encode())
                self._apply_file_record(rec)
                self.rows.extend((file_id, c) for c in chunks)
                self._maybe_train()
                self.version += 1
                self._write_manifest()
            except BaseException:
                self._rollback(first)
                raise
            self._ivf_catch_up()
            self._maybe_screen()
            return file_id, first

    def _rollback(self, first):
        """A failed append: drop this process's uncommitted device rows by re-opening from disk."""
        man, stat = self._read_manifest()
        self.generation = None
        self._sync(man, stat)

    # ---- IVF (config 5) ------------------------------------------------------------------------------
    def _ivf_enabled(self):
        return self.spec.get("kind") == "ivf" and getattr(self.index, "supports_ivf", True)

    def _new_ivf(self):
        nlist = int(self.spec["nlist"])
        if self.ivf_factory is not None:  # injected (host tests)
            return self.ivf_factory(self.dim, nlist, self.device)
        if hasattr(self.index, "new_ivf"):  # row-sharded store: one list set per shard (rfx.sharded)
            return self.index.new_ivf(nlist)
        from .ivf import IvfIndex
        return IvfIndex(self.dim, nlist, self.device)

    def _drop_ivf(self):
        if self.ivf is not None:
            self.ivf.close()
        self.ivf = self.ivf_id = None

    def _live_rows(self):
        ids = [np.arange(f["first"], f["first"] + f["n"], dtype=np.int64)
               for f in self.files.values() if not f["deleted"] and f["n"]]
        return np.sort(np.concatenate(ids)) if ids else np.zeros(0, dtype=np.int64)

    def _maybe_train(self):
        """Writer, under the writer lock, before the manifest commit: train the coarse quantiser
        when the live rows first reach train_min, and again at every 8x growth since the last
        training; the centroids file is fsync'ed before the manifest that names it."""
        if not self._ivf_enabled():
            return
        live = self._live_rows()
        nlist = int(self.spec["nlist"])
        last = self.ivf_meta["rows"] if self.ivf_meta else 0
        if live.size < max(int(self.spec["train_min"]), nlist) or (last and live.size < 8 * last):
            return
        sample = live[::max(1, live.size // (64 * nlist))]
        ivf = self._new_ivf()
        try:
            ivf.train_from(self.index, sample)
            raw = ivf.centroid_bytes()
        except BaseException:
            ivf.close()
            raise
        cid = uuid.uuid4().hex
        hdr = _CENT_MAGIC + np.array([nlist, self.dim, 0], dtype="<u4").tobytes()
        tmp = self._p(f"ivf-{cid}.bin.tmp")
        with open(tmp, "wb") as f:
            f.write(hdr + raw)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self._p(f"ivf-{cid}.bin"))
        _fsync_dir(self.path)
        self._drop_ivf()
        self.ivf, self.ivf_id = ivf, cid  # lists are filled by _ivf_catch_up after the commit
        self.ivf_meta = {"id": cid, "rows": int(live.size)}

    def _ivf_catch_up(self):
        """Bring this process's IVF lists up to the committed rows (caller holds self.lock)."""
        if not self._ivf_enabled() or not self.ivf_meta:
            self._drop_ivf()
            return
        cid = self.ivf_meta["id"]
        if self.ivf_id != cid:
            self._drop_ivf()
            with open(self._p(f"ivf-{cid}.bin"), "rb") as f:
                raw = f.read()
            nlist = int(self.spec["nlist"])
            head = np.frombuffer(raw[8:20], dtype="<u4")
            if raw[:8] != _CENT_MAGIC or int(head[0]) != nlist or int(head[1]) != self.dim \
                    or len(raw) != 20 + nlist * self.dim:
                raise RuntimeError(f"{self.path}: centroid file ivf-{cid}.bin is malformed")
            ivf = self._new_ivf()
            ivf.load_centroids(raw[20:])
            self.ivf, self.ivf_id = ivf, cid
        self.ivf.add_from(self.index, self.index.rows)

    def _maybe_screen(self):
        """Large stores (d 768 / 1024) answer with the exact two-pass scan: an int8
        copy of the rows (dim bytes per row, kept current by every append / tombstone inside librfx)
        screened on the i8 matrix cores (kernel 10: bf16/f16 batches of > 64 questions) or with
        v_dot4 (kernel 11: up to 8 questions, any dtype), the survivors re-scored exactly.
        RFX_SCREEN=auto (default: from RFX_SCREEN_MIN_ROWS rows, 65,536) | 1 (always) | 0 (never).
        Results are the exact scan's either way.
        The copy is an accelerator, never a condition of a write: this runs after the manifest commit
        (and on every reader's catch-up), so it must not raise.  When the copy does not fit
        (RfxCapacityError: device memory minus a reserve, or RFX_SCREEN_MAX_BYTES) or the build fails,
        the store logs it and stays exact; it is not retried for this store generation (the rows only
        grow).  An append that outgrows the copy later is handled inside librfx the same way (the copy
        is dropped, rfx_index_screen_state)."""
        mode = os.environ.get("RFX_SCREEN", "auto")
        if self._screen_on is True:
            # librfx drops the copy when an append outgrows its room (a sharded index drops every shard's,
            # rfx.sharded): that is a state change of the store, not a detail of one index.
            # The store then answers with the exact plan — the same score rule — and does not retry for
            # this generation, as when the copy was declined up front.
            if hasattr(self.index, "screen_state") and self.index.screen_state()[0] == 0:
                self._screen_on = None
                log.warning("store %s: the int8 copy was dropped by growth; answering with the exact scan",
                            self.name)
            return
        if mode == "0" or self._screen_on is not False or not hasattr(self.index, "enable_screen"):
            return
        if self.dtype not in ("bf16", "f16", "f32") or self.dim not in (768, 1024) or self.index.rows == 0:
            return
        if mode != "1" and self.index.rows < int(os.environ.get("RFX_SCREEN_MIN_ROWS", "65536")):
            return
        try:
            self.index.enable_screen(1)
        except (RfxError, RfxTransientError, ValueError) as e:
            # (transient: the index lock was busy — the next catch-up tries again)
            if not isinstance(e, RfxTransientError):
                self._screen_on = None  # declined for this generation: exact scan
            log.warning("store %s: int8 copy not built (%s); answering with the exact scan", self.name, e)
            return
        self._screen_on = True

    def ivf_ready(self) -> bool:
        return self.ivf is not None and self.ivf.rows == self.index.rows

    def delete_file(self, file_id) -> bool:
        with self.lock, self._WriterLock(self):
            self._sync()
            f = self.files.get(file_id)
            if not f or f["deleted"]:
                return False
            try:  # one commit, as in add_document: a failure re-reads the committed state
                if f["n"]:
                    rows = np.arange(f["first"], f["first"] + f["n"], dtype="<i8")
                    self.index.tombstone(rows)
                    _append(self._p("tombs.bin"), 8 * self.tombs, rows.tobytes())
                    self.tombs += len(rows)
                rec = {"op": "del", "id": file_id}
                self.files_bytes = _append(self._p("files.jsonl"), self.files_bytes, (json.dumps(rec) + "\n").encode())
                self._apply_file_record(rec)
                self.version += 1
                self._write_manifest()
            except BaseException:
                self._rollback(None)
                raise
            return True

    # ---- reads -------------------------------------------------------------------------------------
    def tomb_rows(self, start: int, end: int = None) -> np.ndarray:
        """Committed tombstoned rows [start, end) in commit order (tombs.bin; caller holds self.lock):
        what a follower of this store (rfx.union.UnionView) re-applies after a deletion."""
        end = self.tombs if end is None else end
        if end <= start:
            return np.zeros(0, dtype=np.int64)
        return np.frombuffer(_read_range(self._p("tombs.bin"), 8 * start, 8 * end), dtype="<i8").astype(np.int64)

    def search(self, queries, k, row_mask=None):
        """(scores, rows) of the top-k rows per query.  An IVF store with trained lists answers
        unfiltered searches from its lists (nprobe probes, exact re-rank of min(64, max(16, 2k))
        candidates); otherwise, and under a metadata filter, the exact scan runs."""
        if row_mask is None and self.ivf is not None:
            with self.lock:  # the re-rank reads the DeviceIndex rows in place: no append meanwhile
                if self.ivf_ready():
                    s, r = self.ivf.search_index(queries, k, int(self.spec["nprobe"]), self.index,
                                                 rerank_k=min(64, max(16, 2 * int(k))))
                    return s.cpu(), r.cpu()
        return self.index.search(queries, k, row_mask=row_mask)

    def row_mask(self, metadata_filter):
        """Device row mask (int32 words) of the live files whose upload metadata matches the
        filter (rfx.filters), or None when no file matches.  Cached per (store version, filter)."""
        with self.lock:
            key = (self.version, filters.filter_key(metadata_filter))
            if key in self._masks:
                return self._masks[key]
            ranges = self.mask_ranges(metadata_filter)
            mask = None
            if ranges:
                words = filters.row_mask_words(self.index.rows, ranges)
                mask = self.index.mask_tensor(words)
            if len(self._masks) >= 64:
                self._masks.clear()
            self._masks[key] = mask
            return mask

    def mask_ranges(self, metadata_filter):
        """(first, count) row ranges of the live files whose upload metadata matches the filter."""
        with self.lock:
            return [(f["first"], f["n"]) for f in self.files.values()
                    if not f["deleted"] and f["n"] and
                    filters.file_matches(filters.normalize_metadata(f.get("metadata")), metadata_filter)]

    def row_info(self, row):
        """(file_id, chunk text, title, uri) of a row, or None for a row this process has no
        metadata for (cannot happen after a consistent sync; guarded anyway)."""
        if not 0 <= row < len(self.rows):
            return None
        fid, text = self.rows[row]
        f = self.files.get(fid, {})
        return fid, text, f.get("display_name"), f.get("uri")

    def close(self):
        with self.lock:
            self._drop_ivf()
            if self.index is not None:
                self.index.close()


class StoreRegistry:
    """Process-wide map store name -> LocalStore: lazy open, incremental catch-up when another
    process committed, eviction when another process dropped the store."""

    def __init__(self, root=None, device=None, index_factory=None, devices=None, ivf_factory=None):
        """devices (or RFX_DEVICES, e.g. "0,1,2,3,4,5,6,7"; "0x4" = 4 logical shards on device 0):
        more than one -> every store is row-sharded over them (rfx.sharded.ShardedIndex)."""
        self.root = root or default_root()
        self.index_factory = index_factory
        self.device = int(os.environ.get("RFX_DEVICE", "0")) if device is None else int(device)
        spec = devices if devices is not None else os.environ.get("RFX_DEVICES")
        if index_factory is None and spec:
            from .sharded import ShardedIndex, parse_devices
            devs = parse_devices(spec) if isinstance(spec, str) else [int(d) for d in spec]
            if len(devs) > 1:
                self.device = devs[0]
                self.index_factory = lambda dim, dtype, device, _d=tuple(devs): ShardedIndex(dim, dtype, list(_d))
        self.ivf_factory = ivf_factory
        self._stores = {}
        self._lock = threading.Lock()
        self.on_evict = []  # callbacks(name) when a store leaves this registry (rfx.retriever)

    def _dir(self, name):
        if not isinstance(name, str) or not name.startswith(STORE_PREFIX + "local-"):
            return None
        return os.path.join(self.root, name[len(STORE_PREFIX + "local-"):])

    def create(self, display_name, dim, dtype, spec=None):
        """spec: the store's index kind (index_spec_from_env() when None)."""
        name = f"{STORE_PREFIX}local-{uuid.uuid4().hex}"
        os.makedirs(self.root, exist_ok=True)
        st = LocalStore.create(self._dir(name), name, display_name, dim, dtype, self.device, self.index_factory,
                               spec if spec is not None else index_spec_from_env(), self.ivf_factory)
        with self._lock:
            self._stores[name] = st
        return st

    def _evict(self, name):
        st = self._stores.pop(name, None)
        if st is not None:
            st.close()
        for cb in self.on_evict:
            cb(name)

    def get(self, name):
        with self._lock:
            st = self._stores.get(name)
            if st is not None:
                if not st.stale():
                    return st
                if st.refresh():
                    return st
                self._evict(name)  # dropped by another process (cleanup.py delete_store)
                return None
            d = self._dir(name)
            if d is None or not os.path.exists(os.path.join(d, "manifest.json")):
                return None
            try:
                st = LocalStore.open(d, self.device, self.index_factory, self.ivf_factory)
            except StoreGone:
                return None
            self._stores[name] = st
            return st

    def drop(self, name) -> bool:
        with self._lock:
            had = name in self._stores
            self._evict(name)
            d = self._dir(name)
            if d and os.path.isdir(d):
                # the manifest goes first: other processes see the store gone, not half-deleted
                try:
                    os.unlink(os.path.join(d, "manifest.json"))
                except FileNotFoundError:
                    pass
                shutil.rmtree(d, ignore_errors=True)
                return True
            return had

    def names(self):
        out = set(self._stores)
        if os.path.isdir(self.root):
            for d in os.listdir(self.root):
                if os.path.exists(os.path.join(self.root, d, "manifest.json")):
                    out.add(f"{STORE_PREFIX}local-{d}")
        return sorted(out)


_REGISTRY = None
_REG_LOCK = threading.Lock()


def registry() -> StoreRegistry:
    global _REGISTRY
    with _REG_LOCK:
        if _REGISTRY is None:
            _REGISTRY = StoreRegistry()
        return _REGISTRY


def set_registry(reg: StoreRegistry) -> None:
    global _REGISTRY
    with _REG_LOCK:
        _REGISTRY = reg
