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
