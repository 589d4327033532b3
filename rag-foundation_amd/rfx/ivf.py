"""IvfIndex — IVF-Flat int8 index on one device (C ABI rfx_ivf_*, include/rfx.h; kernels
csrc/k_ivf.hip).  SURVEY.md §8 config 5 / build plan item 8: a k-means coarse quantiser, int8
posting lists, a posting-list scan; recall vs brute force < 1 by design.  Every call goes to the
HIP library; there is no CPU path.

Row-sharded multi-GPU use (rfx.dist): train on rank 0, broadcast `centroids()` and call
`set_centroids` on the other ranks, add each rank's rows, then search per rank and merge the
per-rank top-k exactly like the brute-force path (topk_merge_records / gather_merge_records).
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr


class IvfIndex:
    def __init__(self, dim: int, nlist: int, device: int = 0, _handle=None):
        self.dim, self.nlist, self.device = int(dim), int(nlist), int(device)
        if _handle is not None:
            self.handle = _handle
            return
        h = ctypes.c_uint64()
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_create(self.device, self.dim, self.nlist, ctypes.byref(h)))
        self.handle = h.value

    def save(self, path: str) -> None:
        check(lib.rfx_ivf_save(self.handle, path.encode()))

    @classmethod
    def load(cls, path: str, device: int = 0) -> "IvfIndex":
        h = ctypes.c_uint64()
        with torch.cuda.device(device):
            check(lib.rfx_ivf_load(path.encode(), int(device), ctypes.byref(h)))
        dim, nlist = ctypes.c_int(), ctypes.c_int()
        check(lib.rfx_ivf_info(h.value, ctypes.byref(dim), ctypes.byref(nlist), None, None))
        return cls(dim.value, nlist.value, device, _handle=h.value)

    def close(self) -> None:
        if getattr(self, "handle", None):
            check(lib.rfx_ivf_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self):
        return torch.device("cuda", self.device)

    def _rows(self, rows: torch.Tensor):
        if rows.dim() != 2 or rows.shape[1] != self.dim:
            raise ValueError(f"rows must be [n][{self.dim}]")
        dt = {v: k for k, v in _lib.TORCH_DTYPES.items()}.get(rows.dtype)
        if dt is None:
            raise ValueError("rows must be float32, bfloat16 or float16")
        if rows.device != self._dev():
            raise ValueError(f"rows on {rows.device}, index on {self._dev()}")
        return rows.contiguous(), _lib.DTYPE_CODES[dt]

    @property
    def rows(self) -> int:
        n = ctypes.c_int64()
        check(lib.rfx_ivf_info(self.handle, None, None, ctypes.byref(n), None))
        return n.value

    @property
    def trained(self) -> bool:
        t = ctypes.c_int()
        check(lib.rfx_ivf_info(self.handle, None, None, None, ctypes.byref(t)))
        return bool(t.value)

    def train(self, rows: torch.Tensor, iters: int = 10, stream=None) -> None:
        """k-means over sample rows (>= nlist of them)."""
        r, dt = self._rows(rows)
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_train(self.handle, ptr(r), r.shape[0], dt, int(iters), stream_ptr(stream)))

    def centroids(self, stream=None):
        """(int8 [nlist][dim], factors f32 [nlist]) on the device."""
        qc = torch.empty((self.nlist, self.dim), dtype=torch.int8, device=self._dev())
        fc = torch.empty((self.nlist,), dtype=torch.float32, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_get_centroids(self.handle, ptr(qc), ptr(fc), stream_ptr(stream)))
        return qc, fc

    def set_centroids(self, qc: torch.Tensor, stream=None) -> None:
        if qc.dtype != torch.int8 or tuple(qc.shape) != (self.nlist, self.dim) or qc.device != self._dev():
            raise ValueError(f"centroids must be int8 [{self.nlist}][{self.dim}] on {self._dev()}")
        qc = qc.contiguous()
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_set_centroids(self.handle, ptr(qc), stream_ptr(stream)))

    def add(self, rows: torch.Tensor, stream=None) -> int:
        """Quantise + assign rows; returns the first row id."""
        r, dt = self._rows(rows)
        first = self.rows
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_add(self.handle, ptr(r), r.shape[0], dt, stream_ptr(stream)))
        return first

    def build(self, stream=None) -> None:
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_build(self.handle, stream_ptr(stream)))

    def codes(self, stream=None):
        """(codes int8 [rows][dim], inv f32 [rows], labels int32 [rows]) in insertion order."""
        n = self.rows
        c = torch.empty((n, self.dim), dtype=torch.int8, device=self._dev())
        inv = torch.empty((n,), dtype=torch.float32, device=self._dev())
        lab = torch.empty((n,), dtype=torch.int32, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_codes(self.handle, ptr(c), ptr(inv), ptr(lab), stream_ptr(stream)))
        return c, inv, lab

    def lists(self, stream=None):
        """(offsets int64 [nlist+1], row ids int32 [rows] in list order)."""
        off = torch.empty((self.nlist + 1,), dtype=torch.int64, device=self._dev())
        ids = torch.empty((max(self.rows, 1),), dtype=torch.int32, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_lists(self.handle, ptr(off), ptr(ids), stream_ptr(stream)))
        return off, ids[:self.rows]

    def workspace_bytes(self, nq: int, k: int, nprobe: int) -> int:
        b = ctypes.c_size_t()
        check(lib.rfx_ivf_search_workspace_bytes(self.handle, int(nq), int(k), int(nprobe), ctypes.byref(b)))
        return b.value

    def search(self, queries: torch.Tensor, k: int, nprobe: int, workspace: torch.Tensor = None, stream=None):
        """Top-k rows per query over the nprobe nearest lists: (scores f32 [nq][k], rows i64 [nq][k])."""
        q, dt = self._rows(queries)
        nq = q.shape[0]
        out_s = torch.empty((nq, k), dtype=torch.float32, device=self._dev())
        out_r = torch.empty((nq, k), dtype=torch.int64, device=self._dev())
        need = self.workspace_bytes(nq, k, nprobe)
        ws = workspace if workspace is not None and workspace.numel() >= need else \
            torch.empty(max(need, 1), dtype=torch.uint8, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_search(self.handle, ptr(q), nq, dt, int(k), int(nprobe), ptr(out_s), ptr(out_r),
                                     ptr(ws), ws.numel(), stream_ptr(stream)))
        return out_s, out_r

    def search_rerank(self, queries: torch.Tensor, k: int, nprobe: int, rows: torch.Tensor, rerank_k: int = None,
                      stream=None):
        """IVF search keeping rerank_k candidates (default max(k, 16): lists of up to 16 keep the
        fast scan template), re-scored in f32 against the original rows [rows][dim] (insertion
        order, e.g. DeviceIndex.read / the brute-force store)."""
        q, dt = self._rows(queries)
        if rows.dim() != 2 or rows.shape[1] != self.dim or rows.device != self._dev() or not rows.is_contiguous():
            raise ValueError(f"rows must be a contiguous [n][{self.dim}] tensor on {self._dev()}")
        if rows.shape[0] < self.rows:
            raise ValueError(f"rows holds {rows.shape[0]} rows, the index {self.rows}")
        rdt = {v: k_ for k_, v in _lib.TORCH_DTYPES.items()}.get(rows.dtype)
        if rdt is None:
            raise ValueError("rows must be float32, bfloat16 or float16")
        return self._rerank(q, dt, k, nprobe, ptr(rows), _lib.DTYPE_CODES[rdt], rerank_k, stream)

    def _rerank(self, q, dt, k, nprobe, rows_p, rows_code, rerank_k, stream):
        rk = max(int(k), 16) if rerank_k is None else int(rerank_k)
        nq = q.shape[0]
        out_s = torch.empty((nq, k), dtype=torch.float32, device=self._dev())
        out_r = torch.empty((nq, k), dtype=torch.int64, device=self._dev())
        b = ctypes.c_size_t()
        check(lib.rfx_ivf_rerank_workspace_bytes(self.handle, nq, int(k), int(nprobe), rk, ctypes.byref(b)))
        ws = torch.empty(max(b.value, 1), dtype=torch.uint8, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_ivf_search_rerank(self.handle, ptr(q), nq, dt, int(k), int(nprobe), rk, rows_p, rows_code,
                                            ptr(out_s), ptr(out_r), ptr(ws), ws.numel(), stream_ptr(stream)))
        return out_s, out_r

    # ---- serving from a store's DeviceIndex (rfx.store, config 5) ------------------------------------
    def search_index(self, queries: torch.Tensor, k: int, nprobe: int, index, rerank_k: int = None, stream=None):
        """search_rerank against a DeviceIndex holding the same rows in the same order (row i of
        this index = row i of `index`).  Tombstoned rows are NaN there, so the exact re-rank drops
        them.  The caller holds the index owner's lock until the results are read (data_ptr)."""
        q, dt = self._rows(queries)
        if index.dim != self.dim or index.device != self.device:
            raise ValueError("index dim / device differ from the IVF index")
        if index.rows < self.rows:
            raise ValueError(f"index holds {index.rows} rows, the IVF lists {self.rows}")
        return self._rerank(q, dt, k, nprobe, ctypes.c_void_p(index.data_ptr()), _lib.DTYPE_CODES[index.dtype],
                            rerank_k, stream)

    def train_from(self, index, row_ids, iters: int = 10) -> None:
        """k-means over the rows `row_ids` (sorted int64 numpy array) of a DeviceIndex."""
        import numpy as np
        ids = np.asarray(row_ids, dtype=np.int64)
        parts, span = [], 1 << 20
        for r0 in range(0, int(ids[-1]) + 1 if ids.size else 0, span):
            sel = ids[(ids >= r0) & (ids < r0 + span)] - r0
            if sel.size:
                m = int(sel[-1]) + 1
                parts.append(index.read(r0, m)[torch.from_numpy(sel).to(self._dev())])
        self.train(torch.cat(parts) if parts else torch.empty((0, self.dim), device=self._dev()), iters)

    def add_from(self, index, upto: int) -> None:
        """Assign rows [self.rows, upto) of a DeviceIndex to their lists (1M-row pieces)."""
        span = 1 << 20
        while self.rows < upto:
            r0 = self.rows
            self.add(index.read(r0, min(span, upto - r0)))

    def centroid_bytes(self) -> bytes:
        return self.centroids()[0].cpu().numpy().tobytes()

    def load_centroids(self, raw: bytes) -> None:
        import numpy as np
        qc = np.frombuffer(raw, dtype=np.int8).reshape(self.nlist, self.dim)
        self.set_centroids(torch.from_numpy(qc.copy()).to(self._dev()))


def rerank_candidates(queries: torch.Tensor, rows_ptr: int, rows_dtype: str, row_lo: int, n_rows: int,
                      cand: torch.Tensor, stream=None):
    """Exact f32 re-score of global candidate rows cand [nq][n_cand] (int64, < 0 = padding) against
    one shard's rows (device pointer to [n_rows][dim] of rows_dtype holding global rows
    [row_lo, row_lo + n_rows)); candidates outside the shard come back (-inf, -1).
    -> (scores f32 [nq][n_cand], rows int64 [nq][n_cand]) (rfx_rerank_candidates)."""
    dt = {v: k for k, v in _lib.TORCH_DTYPES.items()}.get(queries.dtype)
    if dt is None or queries.dim() != 2 or not queries.is_cuda:
        raise ValueError("queries must be a cuda float32/bfloat16/float16 [nq][dim] tensor")
    if cand.dtype != torch.int64 or cand.dim() != 2 or cand.shape[0] != queries.shape[0] or cand.device != queries.device:
        raise ValueError("candidates must be int64 [nq][n_cand] on the queries' device")
    q, c = queries.contiguous(), cand.contiguous()
    nq, nc = c.shape
    out_s = torch.empty((nq, nc), dtype=torch.float32, device=q.device)
    out_r = torch.empty((nq, nc), dtype=torch.int64, device=q.device)
    with torch.cuda.device(q.device):
        check(lib.rfx_rerank_candidates(ptr(q), nq, _lib.DTYPE_CODES[dt], ctypes.c_void_p(int(rows_ptr)),
                                        _lib.DTYPE_CODES[rows_dtype], int(row_lo), int(n_rows), q.shape[1], ptr(c),
                                        nc, ptr(out_s), ptr(out_r), stream_ptr(stream)))
    return out_s, out_r


def quantize(rows: torch.Tensor, stream=None):
    """int8 codes [n][dim] + inv scales [n] of rows (the IVF code format)."""
    dt = {v: k for k, v in _lib.TORCH_DTYPES.items()}[rows.dtype]
    rows = rows.contiguous()
    n, d = rows.shape
    codes = torch.empty((n, d), dtype=torch.int8, device=rows.device)
    inv = torch.empty((n,), dtype=torch.float32, device=rows.device)
    with torch.cuda.device(rows.device):
        check(lib.rfx_quantize(ptr(rows), n, d, _lib.DTYPE_CODES[dt], ptr(codes), ptr(inv), stream_ptr(stream)))
    return codes, inv


def synth_clustered(cseed: int, ncenters: int, seed: int, row0: int, n: int, dim: int, dtype: str = "bf16",
                    device: int = 0) -> torch.Tensor:
    """Clustered synthetic rows on the device (oracle/ivf.py clustered_rows)."""
    out = torch.empty((n, dim), dtype=_lib.TORCH_DTYPES[dtype], device=torch.device("cuda", device))
    with torch.cuda.device(device):
        check(lib.rfx_synth_clustered(ctypes.c_uint64(cseed), int(ncenters), ctypes.c_uint64(seed), int(row0), int(n),
                                      int(dim), _lib.DTYPE_CODES[dtype], ptr(out), stream_ptr()))
    return out
