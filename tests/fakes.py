"""Test-only retriever backed by the CPU oracle (lets the adapter's host logic be tested on a
machine without a GPU).  Never used by the product: LocalGpuRag defaults to GpuRetriever."""
import uuid

import numpy as np

from oracle import embed as oembed
from oracle import search as osearch
from oracle import synth as osynth
from oracle import textproc
from rfx import filters
from rfx.retriever import Hit, _chunking

V, DIM = 4096, 768
W_SEED, H_SEED = 0x5241475F454D4244, 0x5241475F544F4B4E


class OracleRetriever:
    def __init__(self, dim=DIM):
        self.dim = dim
        self.wt = oembed.weights_int(V, dim, W_SEED)
        self.stores = {}

    def create_store(self, display_name):
        name = f"fileSearchStores/local-{uuid.uuid4().hex}"
        self.stores[name] = {"rows": [], "vecs": np.zeros((0, self.dim)), "files": {}}
        return name

    def drop_store(self, name):
        return self.stores.pop(name, None) is not None

    def store_names(self):
        return sorted(self.stores)

    def _embed(self, texts):
        b = [t.lower().encode() for t in texts]
        raw = b"".join(b)
        offs = np.cumsum([0] + [len(x) for x in b])
        csr = textproc.featurize(raw, list(zip(offs[:-1], offs[1:])), V, H_SEED)
        return oembed.embed(*csr, V, self.wt, "f32").astype(np.float64)

    def add_document(self, store_name, text, display_name, chunking_config=None, metadata=None):
        st = self.stores.get(store_name)
        if st is None:
            raise ValueError(f"unknown store {store_name!r}")
        mt, ov = _chunking(chunking_config)
        raw = text.encode()
        chunks = [raw[s:e].decode() for s, e in textproc.chunk_whitespace(raw, mt, ov)]
        fid = f"files/local-{uuid.uuid4().hex}"
        first = len(st["rows"])
        st["rows"] += [(fid, c) for c in chunks]
        st["vecs"] = np.concatenate([st["vecs"], self._embed(chunks)]) if chunks else st["vecs"]
        st["files"][fid] = {"first": first, "n": len(chunks), "title": display_name, "metadata": metadata}
        return fid, len(chunks)

    def delete_file(self, store_name, file_id):
        st = self.stores.get(store_name)
        f = st and st["files"].get(file_id)
        if not f:
            return False
        st["vecs"][f["first"]:f["first"] + f["n"]] = np.nan
        return True

    def search(self, store_names, question, k, metadata_filter=None):
        if not 1 <= int(k) <= 64:
            raise ValueError(f"top_k={k} out of range [1, 64]")
        filt = filters.check_filter(metadata_filter)
        hits = []
        q = self._embed([question])
        for si, name in enumerate(store_names or []):
            st = self.stores.get(name)
            if not st or not st["rows"]:
                continue
            vecs = st["vecs"]
            if filt is not None:  # rows of non-matching files are excluded (NaN, the tombstone rule)
                keep = np.zeros(len(vecs), dtype=bool)
                for f in st["files"].values():
                    if filters.file_matches(filters.normalize_metadata(f["metadata"]), filt):
                        keep[f["first"]:f["first"] + f["n"]] = True
                vecs = np.where(keep[:, None], vecs, np.nan)
            s, r = osearch.topk(q, vecs, k)
            for sc, row in zip(s[0], r[0]):
                if row < 0:
                    continue
                fid, text = st["rows"][row]
                title = st["files"][fid]["title"]
                hits.append((-sc, si, row, Hit(float(sc), name, int(row), fid, text, title, f"local://{name}/{fid}")))
        hits.sort(key=lambda h: h[:3])
        return [h[3] for h in hits[:k]]


class HostIndex:
    """Test-only host stand-in for rfx.index.DeviceIndex, with the same interface LocalStore
    uses and the same append-only row-file format as rfx_rows_append / rfx_rows_sync (64-byte
    header "RFXROWS1", u32 version 1, u32 dim, u32 dtype; row-major rows).  Lets the store's file
    protocol (commit point, torn tails, cross-process catch-up, writer lock) run on a CPU."""

    CODES = {"f32": (0, np.float32), "bf16": (1, np.uint16), "f16": (2, np.float16)}
    syncs = []  # (path, rows before, upto) of every rows_sync, for the incremental-load tests

    def __init__(self, dim, dtype="f32", device=0, capacity=0):
        self.dim, self.dtype, self.device = int(dim), dtype, device
        self.code, self.np_dtype = self.CODES[dtype]
        self.data = np.zeros((0, self.dim), dtype=self.np_dtype)
        self.closed = False

    def _hdr(self):
        h = bytearray(64)
        h[:8] = b"RFXROWS1"
        h[8:20] = np.array([1, self.dim, self.code], dtype="<u4").tobytes()
        return bytes(h)

    @property
    def rows(self):
        return self.data.shape[0]

    def add(self, vecs):
        v = np.asarray(vecs, dtype=self.np_dtype).reshape(-1, self.dim)
        first = self.rows
        self.data = np.concatenate([self.data, v])
        return first

    def rows_append(self, path, row0):
        import os
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            if os.fstat(fd).st_size >= 64:
                assert os.pread(fd, 64, 0) == self._hdr()
            else:
                assert row0 == 0
                os.pwrite(fd, self._hdr(), 0)
            rb = self.dim * self.data.itemsize
            assert os.fstat(fd).st_size >= 64 + row0 * rb, "row file shorter than the append point"
            os.ftruncate(fd, 64 + row0 * rb)
            os.pwrite(fd, self.data[row0:].tobytes(), 64 + row0 * rb)
            os.fsync(fd)
        finally:
            os.close(fd)

    def rows_sync(self, path, upto):
        HostIndex.syncs.append((path, self.rows, upto))
        rb = self.dim * self.data.itemsize
        with open(path, "rb") as f:
            assert f.read(64) == self._hdr()
            f.seek(64 + self.rows * rb)
            raw = f.read((upto - self.rows) * rb)
        assert len(raw) == (upto - self.rows) * rb, "row file shorter than the committed count"
        self.data = np.concatenate([self.data, np.frombuffer(raw, dtype=self.np_dtype).reshape(-1, self.dim)])

    def tombstone(self, rows):
        rows = np.asarray(rows, dtype=np.int64)
        self.data = self.data.copy()
        self.data[rows] = np.nan if self.dtype != "bf16" else 0x7FC0

    def mask_tensor(self, words):
        return words

    def close(self):
        self.closed = True

    def read(self, row0, n):
        """Rows [row0, row0 + n) decoded to f32 (NaN for tombstoned rows)."""
        d = self.data[row0:row0 + n]
        if self.dtype == "bf16":
            return (d.astype(np.uint32) << 16).view(np.float32)
        return d.astype(np.float32)


class HostIvf:
    """Test-only host stand-in for rfx.ivf.IvfIndex with the interface LocalStore uses (train_from,
    centroid_bytes / load_centroids, add_from, search_index).  The quantiser is deliberately
    simple (centroids = the first nlist sampled rows, int8); what the store tests check is the
    protocol around it: who trains, which centroids every process loads, that lists grow by the
    appended rows only, and that the re-rank reads the store's rows (tombstones NaN)."""

    log = []  # (op, args) of every call, for the protocol tests

    def __init__(self, dim, nlist, device=0):
        self.dim, self.nlist = int(dim), int(nlist)
        self.qc = None
        self.labels = np.zeros(0, dtype=np.int64)
        self.closed = False

    @property
    def rows(self):
        return self.labels.size

    @staticmethod
    def _q8(x):
        a = np.nanmax(np.abs(x), axis=1, keepdims=True)
        a = np.where(np.isfinite(a) & (a > 0), a, 1.0)
        return np.clip(np.rint(np.nan_to_num(x) * (127.0 / a)), -127, 127).astype(np.int8)

    def train_from(self, index, row_ids):
        HostIvf.log.append(("train", len(row_ids)))
        x = index.read(0, index.rows)[np.asarray(row_ids)]
        assert not np.isnan(x).any(), "training sample holds tombstoned rows"
        self.qc = self._q8(x[:self.nlist])

    def centroid_bytes(self):
        return self.qc.tobytes()

    def load_centroids(self, raw):
        HostIvf.log.append(("load", len(raw)))
        self.qc = np.frombuffer(raw, dtype=np.int8).reshape(self.nlist, self.dim).copy()

    def add_from(self, index, upto):
        if upto > self.rows:
            HostIvf.log.append(("add", self.rows, upto))
            x = self._q8(index.read(self.rows, upto - self.rows)).astype(np.int64)
            self.labels = np.concatenate([self.labels, np.argmax(x @ self.qc.astype(np.int64).T, axis=1)])

    def search_index(self, queries, k, nprobe, index, rerank_k=None):
        import torch
        q = np.asarray(queries, dtype=np.float32)
        x = index.read(0, self.rows)
        out_s = np.full((len(q), k), -np.inf, dtype=np.float32)
        out_r = np.full((len(q), k), -1, dtype=np.int64)
        for i, qi in enumerate(q):
            probe = np.argsort(-(self.qc.astype(np.float32) @ qi), kind="stable")[:nprobe]
            cand = np.flatnonzero(np.isin(self.labels, probe))
            sc = x[cand] @ qi
            keep = ~np.isnan(sc)
            cand, sc = cand[keep], sc[keep]
            order = np.lexsort((cand, -sc))[:k]
            out_s[i, :len(order)], out_r[i, :len(order)] = sc[order], cand[order]
        return torch.from_numpy(out_s), torch.from_numpy(out_r)

    def close(self):
        self.closed = True
