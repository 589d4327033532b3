"""Chunker + embedder of the index write (upload_file, gemini_rag.py:307-352) and of the query
(ask_stream, gemini_rag.py:517-551), which the reference leaves to Gemini File Search.

Host (C, csrc/featurize.cpp): whitespace chunking (Gemini white_space_config semantics) and the
reference tokeniser (scripts/benchmark/metrics.py:13-19) restated on bytes, hashed into V signed
buckets.  Device (HIP, csrc/k_embed.hip): densify + MFMA contraction with the seeded projection +
exact L2 normalisation, written straight in the index dtype.
"""
import ctypes
import threading

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr

DEFAULT_V = 4096
DEFAULT_DIM = 768
DEFAULT_W_SEED = 0x5241475F454D4244  # "RAG_EMBD"
DEFAULT_HASH_SEED = 0x5241475F544F4B4E  # "RAG_TOKN"
# Gemini File Search's documented white_space_config example values (the reference forwards
# chunking_config unchanged, gemini_rag.py:324-326).
DEFAULT_MAX_TOKENS = 200
DEFAULT_OVERLAP = 20

_W_CACHE = {}
_W_LOCK = threading.Lock()


def prep_text(text: str) -> bytes:
    """UTF-8 bytes for the byte-level tokeniser: non-ASCII text gets Python's str.lower() first
    (the only Unicode-sensitive step of metrics._normalize)."""
    return text.encode("utf-8") if text.isascii() else text.lower().encode("utf-8")


def chunk_spans(raw: bytes, max_tokens: int = DEFAULT_MAX_TOKENS, overlap: int = DEFAULT_OVERLAP):
    """Whitespace windows over raw bytes -> int64 array [n][2] of (start, end) byte offsets."""
    n = ctypes.c_int64()
    buf = ctypes.create_string_buffer(raw, len(raw)) if raw else None
    check(lib.rfx_chunk_whitespace(buf, len(raw), int(max_tokens), int(overlap), None, 0, ctypes.byref(n)),
          "chunking config")
    spans = np.zeros((n.value, 2), dtype=np.int64)
    if n.value:
        check(lib.rfx_chunk_whitespace(buf, len(raw), int(max_tokens), int(overlap), spans.ctypes.data, n.value,
                                       ctypes.byref(n)))
    return spans


def featurize(raw: bytes, spans: np.ndarray, V: int = DEFAULT_V, hash_seed: int = DEFAULT_HASH_SEED):
    """CSR hashed features (indptr int32 [n+1], bucket int32 [nnz], count int16 [nnz])."""
    spans = np.ascontiguousarray(spans, dtype=np.int64).reshape(-1, 2)
    n = spans.shape[0]
    indptr = np.zeros(n + 1, dtype=np.int32)
    buf = ctypes.create_string_buffer(raw, len(raw)) if raw else ctypes.create_string_buffer(1)
    nnz = ctypes.c_int64()
    check(lib.rfx_featurize(buf, spans.ctypes.data, n, int(V), ctypes.c_uint64(hash_seed), indptr.ctypes.data,
                            None, None, 0, ctypes.byref(nnz)), "featurize")
    bucket = np.zeros(max(nnz.value, 1), dtype=np.int32)
    count = np.zeros(max(nnz.value, 1), dtype=np.int16)
    check(lib.rfx_featurize(buf, spans.ctypes.data, n, int(V), ctypes.c_uint64(hash_seed), indptr.ctypes.data,
                            bucket.ctypes.data, count.ctypes.data, nnz.value, ctypes.byref(nnz)), "featurize")
    return indptr, bucket[:nnz.value], count[:nnz.value]


def featurize_texts(texts, V: int = DEFAULT_V, hash_seed: int = DEFAULT_HASH_SEED):
    """One chunk per text (queries, or chunks that need per-chunk str.lower())."""
    parts = [prep_text(t) for t in texts]
    raw = b"".join(parts)
    offs = np.cumsum([0] + [len(p) for p in parts])
    spans = np.stack([offs[:-1], offs[1:]], axis=1) if parts else np.zeros((0, 2), np.int64)
    return featurize(raw, spans, V, hash_seed)


class Embedder:
    """Seeded hashed-feature projection embedder (V buckets -> dim), resident on one device."""

    def __init__(self, dim: int = DEFAULT_DIM, V: int = DEFAULT_V, seed: int = DEFAULT_W_SEED,
                 hash_seed: int = DEFAULT_HASH_SEED, device: int = 0):
        self.dim, self.V, self.seed, self.hash_seed, self.device = int(dim), int(V), int(seed), int(hash_seed), int(device)

    @property
    def weights(self) -> torch.Tensor:
        key = (self.V, self.dim, self.seed, self.device)
        with _W_LOCK:
            w = _W_CACHE.get(key)
            if w is None:
                w = torch.empty((self.dim, self.V), dtype=torch.bfloat16, device=torch.device("cuda", self.device))
                with torch.cuda.device(self.device):
                    check(lib.rfx_embed_weights(self.V, self.dim, ctypes.c_uint64(self.seed), ptr(w), stream_ptr()))
                _W_CACHE[key] = w
            return w

    def embed_csr(self, indptr, bucket, count, dtype: str = "bf16") -> torch.Tensor:
        n = len(indptr) - 1
        dev = torch.device("cuda", self.device)
        out = torch.empty((n, self.dim), dtype=_lib.TORCH_DTYPES[dtype], device=dev)
        if n == 0:
            return out
        ip = torch.from_numpy(np.ascontiguousarray(indptr)).to(dev)
        bk = torch.from_numpy(np.ascontiguousarray(bucket) if len(bucket) else np.zeros(1, np.int32)).to(dev)
        ct = torch.from_numpy(np.ascontiguousarray(count) if len(count) else np.zeros(1, np.int16)).to(dev)
        wsb = ctypes.c_size_t()
        check(lib.rfx_embed_workspace_bytes(n, self.V, ctypes.byref(wsb)))
        ws = torch.empty(max(wsb.value, 1), dtype=torch.uint8, device=dev)
        w = self.weights
        with torch.cuda.device(self.device):
            check(lib.rfx_embed(ptr(ip), ptr(bk), ptr(ct), n, self.V, ptr(w), self.dim, ptr(out),
                                _lib.DTYPE_CODES[dtype], ptr(ws), ws.numel(), stream_ptr()))
        return out

    def embed_texts(self, texts, dtype: str = "bf16") -> torch.Tensor:
        return self.embed_csr(*featurize_texts(texts, self.V, self.hash_seed), dtype=dtype)

    def chunk_and_embed(self, text: str, dtype: str = "bf16", max_tokens: int = DEFAULT_MAX_TOKENS,
                        overlap: int = DEFAULT_OVERLAP):
        """Chunk a document and embed every chunk -> (chunk texts, [n][dim] tensor)."""
        raw = text.encode("utf-8")
        spans = chunk_spans(raw, max_tokens, overlap)
        chunks = [raw[s:e].decode("utf-8", errors="replace") for s, e in spans]
        if text.isascii():
            csr = featurize(raw, spans, self.V, self.hash_seed)
        else:
            csr = featurize_texts(chunks, self.V, self.hash_seed)
        return chunks, self.embed_csr(*csr, dtype=dtype)
