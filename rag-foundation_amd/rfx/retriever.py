"""GpuRetriever — the index-write / search engine behind LocalGpuRag.

Every call goes to the HIP library (librfx.so); there is no CPU path.
"""
import os
import threading
from dataclasses import dataclass

import torch

from .embedder import DEFAULT_MAX_TOKENS, DEFAULT_OVERLAP, Embedder
from .store import registry as default_registry


@dataclass
class Hit:
    score: float
    store: str
    row: int
    file_id: str
    text: str
    title: str
    uri: str


def _chunking(cfg):
    """Gemini chunking_config -> (max_tokens, overlap); defaults when absent."""
    if not cfg:
        return DEFAULT_MAX_TOKENS, DEFAULT_OVERLAP
    ws = cfg.get("white_space_config", cfg) if isinstance(cfg, dict) else {}
    mt = int(ws.get("max_tokens_per_chunk", DEFAULT_MAX_TOKENS))
    ov = int(ws.get("max_overlap_tokens", DEFAULT_OVERLAP))
    return mt, min(ov, mt - 1)


class GpuRetriever:
    def __init__(self, registry=None, dim=None, dtype=None):
        self._registry = registry
        self.dim = int(os.environ.get("RFX_DIM", "768")) if dim is None else int(dim)
        self.dtype = os.environ.get("RFX_DTYPE", "f32") if dtype is None else dtype
        self._emb = {}
        self._lock = threading.Lock()

    @property
    def registry(self):
        return self._registry or default_registry()

    def embedder(self, dim) -> Embedder:
        with self._lock:
            e = self._emb.get(dim)
            if e is None:
                e = Embedder(dim=dim, device=self.registry.device)
                self._emb[dim] = e
            return e

    # ---- store namespace ----------------------------------------------------------------------
    def create_store(self, display_name):
        return self.registry.create(display_name, self.dim, self.dtype).name

    def drop_store(self, name):
        return self.registry.drop(name)

    def store_names(self):
        return self.registry.names()

    # ---- index write --------------------------------------------------------------------------
    def add_document(self, store_name, text, display_name, chunking_config=None, metadata=None):
        st = self.registry.get(store_name)
        if st is None:
            raise ValueError(f"unknown store {store_name!r}")
        mt, ov = _chunking(chunking_config)
        with torch.cuda.device(st.device):
            chunks, vecs = self.embedder(st.dim).chunk_and_embed(text, st.dtype, mt, ov)
            file_id, _ = st.add_document(chunks, vecs, display_name, metadata)
        return file_id, len(chunks)

    def delete_file(self, store_name, file_id):
        st = self.registry.get(store_name)
        return bool(st and st.delete_file(file_id))

    # ---- retrieval ----------------------------------------------------------------------------
    def search(self, store_names, question, k):
        """Top-k hits over the union of the named stores, rank order (score desc, store order,
        row asc)."""
        hits = []
        for si, name in enumerate(store_names or []):
            st = self.registry.get(name)
            if st is None or st.index.rows == 0:
                continue
            with torch.cuda.device(st.device):
                q = self.embedder(st.dim).embed_texts([question], st.dtype)
                s, r = st.index.search(q, k)
                s, r = s.cpu().tolist()[0], r.cpu().tolist()[0]
            for sc, row in zip(s, r):
                if row < 0:
                    continue
                fid, text, title, uri = st.row_info(row)
                hits.append((-sc, si, row, Hit(sc, name, row, fid, text, title, uri)))
        hits.sort(key=lambda h: h[:3])
        return [h[3] for h in hits[:k]]
