"""Local File-Search-store equivalent: a DeviceIndex plus per-row chunk metadata, persisted on
disk so that the API processes can serve what the ingestion worker wrote (the worker deletes the
uploaded file after indexing, backend/app/services/ingestion.py:341).

On-disk layout of a store (directory <root>/<store id>/):
  manifest.json   {"name", "display_name", "dim", "dtype", "version", "files": {file_id: {...}}}
  index.rfx       rfx_index_save() image (rows + tombstones)
  meta.jsonl      one JSON object per row: {"f": file_id, "t": chunk text}
GPU state is a process-level singleton (StoreRegistry), because get_rag_client() builds a new
adapter per request (chat.py:937, ingestion.py:214).
"""
import json
import os
import shutil
import threading
import uuid

import torch

from . import filters
from .index import DeviceIndex

STORE_PREFIX = "fileSearchStores/"  # accepted by routes/stores.py:46 (prefix check)


def default_root() -> str:
    return os.environ.get("RFX_INDEX_DIR", os.path.join(os.path.expanduser("~"), ".cache", "rfx", "stores"))


class LocalStore:
    def __init__(self, name, display_name, dim, dtype, device, path):
        self.name, self.display_name = name, display_name
        self.dim, self.dtype, self.device, self.path = dim, dtype, device, path
        self.index = DeviceIndex(dim, dtype, device)
        self.rows = []      # per row: (file_id, chunk text)
        self.files = {}     # file_id -> {"first", "n", "display_name", "uri", "deleted", "metadata"}
        self.version = 0
        self.lock = threading.RLock()
        self._mtime = None
        self._masks = {}    # (version, filter key) -> device row mask

    # ---- persistence ------------------------------------------------------------------------
    def _manifest(self):
        return {"name": self.name, "display_name": self.display_name, "dim": self.dim, "dtype": self.dtype,
                "version": self.version, "rows": len(self.rows), "files": self.files}

    def save(self):
        os.makedirs(self.path, exist_ok=True)
        self.index.save(os.path.join(self.path, "index.rfx"))
        tmp = os.path.join(self.path, "meta.jsonl.tmp")
        with open(tmp, "w", encoding="utf-8") as f:
            for fid, text in self.rows:
                f.write(json.dumps({"f": fid, "t": text}, ensure_ascii=False) + "\n")
        os.replace(tmp, os.path.join(self.path, "meta.jsonl"))
        tmp = os.path.join(self.path, "manifest.json.tmp")
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(self._manifest(), f)
        os.replace(tmp, os.path.join(self.path, "manifest.json"))
        self._mtime = os.stat(os.path.join(self.path, "manifest.json")).st_mtime_ns

    @classmethod
    def load(cls, path, device):
        with open(os.path.join(path, "manifest.json"), encoding="utf-8") as f:
            man = json.load(f)
        st = cls.__new__(cls)
        st.name, st.display_name = man["name"], man["display_name"]
        st.dim, st.dtype, st.device, st.path = man["dim"], man["dtype"], device, path
        st.version = man["version"]
        st.files = man["files"]
        st.lock = threading.RLock()
        st._masks = {}
        idx = os.path.join(path, "index.rfx")
        st.index = DeviceIndex.load(idx, device) if os.path.exists(idx) else DeviceIndex(st.dim, st.dtype, device)
        st.rows = []
        meta = os.path.join(path, "meta.jsonl")
        if os.path.exists(meta):
            with open(meta, encoding="utf-8") as f:
                for line in f:
                    o = json.loads(line)
                    st.rows.append((o["f"], o["t"]))
        st._mtime = os.stat(os.path.join(path, "manifest.json")).st_mtime_ns
        return st

    def stale(self) -> bool:
        try:
            return os.stat(os.path.join(self.path, "manifest.json")).st_mtime_ns != self._mtime
        except FileNotFoundError:
            return False

    # ---- writes ------------------------------------------------------------------------------
    def add_document(self, chunks, vecs, display_name, metadata=None):
        with self.lock:
            file_id = f"files/local-{uuid.uuid4().hex}"
            first = self.index.add(vecs) if len(chunks) else self.index.rows
            for c in chunks:
                self.rows.append((file_id, c))
            self.files[file_id] = {"first": first, "n": len(chunks), "display_name": display_name,
                                   "uri": f"local://{self.name}/{file_id}", "deleted": False,
                                   "metadata": metadata or None}
            self.version += 1
            self.save()
            return file_id, first

    def delete_file(self, file_id) -> bool:
        with self.lock:
            f = self.files.get(file_id)
            if not f or f["deleted"]:
                return False
            if f["n"]:
                self.index.tombstone(range(f["first"], f["first"] + f["n"]))
            f["deleted"] = True
            self.version += 1
            self.save()
            return True

    def row_mask(self, metadata_filter):
        """Device row mask (int32 words) of the live files whose upload metadata matches the
        filter (rfx.filters), or None when no file matches.  Cached per (store version, filter)."""
        key = (self.version, filters.filter_key(metadata_filter))
        with self.lock:
            if key in self._masks:
                return self._masks[key]
            ranges = [(f["first"], f["n"]) for f in self.files.values()
                      if not f["deleted"] and f["n"] and
                      filters.file_matches(filters.normalize_metadata(f.get("metadata")), metadata_filter)]
            mask = None
            if ranges:
                words = filters.row_mask_words(self.index.rows, ranges)
                mask = torch.from_numpy(words).to(f"cuda:{self.device}")
            if len(self._masks) >= 64:
                self._masks.clear()
            self._masks[key] = mask
            return mask

    def row_info(self, row):
        fid, text = self.rows[row]
        f = self.files.get(fid, {})
        return fid, text, f.get("display_name"), f.get("uri")


class StoreRegistry:
    """Process-wide map store name -> LocalStore (lazy load, reload when another process wrote)."""

    def __init__(self, root=None, device=None):
        self.root = root or default_root()
        self.device = int(os.environ.get("RFX_DEVICE", "0")) if device is None else int(device)
        self._stores = {}
        self._lock = threading.Lock()

    def _dir(self, name):
        if not isinstance(name, str) or not name.startswith(STORE_PREFIX + "local-"):
            return None
        return os.path.join(self.root, name[len(STORE_PREFIX + "local-"):])

    def create(self, display_name, dim, dtype):
        name = f"{STORE_PREFIX}local-{uuid.uuid4().hex}"
        st = LocalStore(name, display_name, dim, dtype, self.device, self._dir(name))
        st.save()
        with self._lock:
            self._stores[name] = st
        return st

    def get(self, name):
        with self._lock:
            st = self._stores.get(name)
            if st is not None and not st.stale():
                return st
            d = self._dir(name)
            if d is None or not os.path.exists(os.path.join(d, "manifest.json")):
                return None
            st = LocalStore.load(d, self.device)
            self._stores[name] = st
            return st

    def drop(self, name) -> bool:
        with self._lock:
            st = self._stores.pop(name, None)
            if st is not None:
                st.index.close()
            d = self._dir(name)
            if d and os.path.isdir(d):
                shutil.rmtree(d, ignore_errors=True)
                return True
            return st is not None

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
