"""DeviceIndex — one vector-store shard resident in HBM (wrapper over an rfx_index_t handle).

This is the vector store behind a File Search store name (GeminiRag.create_store,
backend/app/services/gemini_rag.py:271-304) and the target of the index write
(upload_file, gemini_rag.py:307-352) and of retrieval (ask_stream, gemini_rag.py:517-551).
Layout in HBM: row-major [capacity][dim] of the index dtype (f32 / bf16 / f16).
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr


class DeviceIndex:
    def __init__(self, dim: int, dtype: str = "bf16", device: int = 0, capacity: int = 0, _handle=None):
        if dtype not in _lib.DTYPE_CODES:
            raise ValueError(f"dtype must be one of {list(_lib.DTYPE_CODES)}")
        self.dim = int(dim)
        self.dtype = dtype
        self.device = int(device)
        if _handle is not None:
            self.handle = _handle
        else:
            h = ctypes.c_uint64()
            check(lib.rfx_index_create(self.device, self.dim, _lib.DTYPE_CODES[dtype], int(capacity), ctypes.byref(h)))
            self.handle = h.value

    # ---- lifecycle ----------------------------------------------------------------------------
    @classmethod
    def load(cls, path: str, device: int = 0) -> "DeviceIndex":
        h = ctypes.c_uint64()
        check(lib.rfx_index_load(path.encode(), int(device), ctypes.byref(h)))
        dim, dt = ctypes.c_int(), ctypes.c_int()
        check(lib.rfx_index_info(h.value, ctypes.byref(dim), ctypes.byref(dt), None, None, None))
        name = {v: k for k, v in _lib.DTYPE_CODES.items()}[dt.value]
        return cls(dim.value, name, device, _handle=h.value)

    def save(self, path: str) -> None:
        check(lib.rfx_index_save(self.handle, path.encode()))

    def rows_append(self, path: str, row0: int, file_base: int = 0) -> None:
        """Write rows [row0, rows) to the store's append-only row file (fsync'ed); index row i is
        file row file_base + i."""
        with torch.cuda.device(self.device):
            check(lib.rfx_rows_append(self.handle, path.encode(), int(row0), int(file_base)))

    def rows_sync(self, path: str, upto: int, file_base: int = 0) -> None:
        """Append file rows [file_base + rows, file_base + upto) written by another process."""
        with torch.cuda.device(self.device):
            check(lib.rfx_rows_sync(self.handle, path.encode(), int(upto), int(file_base)))

    def data_ptr(self) -> int:
        """Device address of row 0 (rows contiguous, row-major, tombstoned rows NaN).  Valid until
        the next add / reserve / rows_sync, which may reallocate: the owner's lock must be held
        across every use (rfx.store.LocalStore.search)."""
        p = ctypes.c_void_p()
        check(lib.rfx_index_data(self.handle, ctypes.byref(p)))
        return p.value

    def mask_tensor(self, words):
        """Row-mask words (numpy int32) as the device tensor the masked search takes."""
        return torch.from_numpy(words).to(self._dev())

    def close(self) -> None:
        if getattr(self, "handle", None):
            check(lib.rfx_index_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- info ---------------------------------------------------------------------------------
    def _info(self):
        rows, cap, live = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib.rfx_index_info(self.handle, None, None, ctypes.byref(rows), ctypes.byref(cap), ctypes.byref(live)))
        return rows.value, cap.value, live.value

    @property
    def rows(self) -> int:
        return self._info()[0]

    @property
    def capacity(self) -> int:
        """Rows the device buffer holds (rows beyond `rows` are NaN); a union view maps members whole."""
        return self._info()[1]

    @property
    def live_rows(self) -> int:
        return self._info()[2]

    @property
    def torch_dtype(self):
        return _lib.TORCH_DTYPES[self.dtype]

    def _dev(self):
        return torch.device("cuda", self.device)

    # ---- writes -------------------------------------------------------------------------------
    def reserve(self, capacity: int) -> None:
        check(lib.rfx_index_reserve(self.handle, int(capacity)))

    def add(self, vecs: torch.Tensor) -> int:
        """Append normalised rows [n][dim] of the index dtype (device or host tensor)."""
        if vecs.dim() != 2 or vecs.shape[1] != self.dim:
            raise ValueError(f"expected [n][{self.dim}] rows, got {tuple(vecs.shape)}")
        if vecs.dtype != self.torch_dtype:
            raise ValueError(f"expected {self.torch_dtype} rows, got {vecs.dtype}")
        vecs = vecs.contiguous()
        first = ctypes.c_int64()
        on_dev = vecs.is_cuda
        st = stream_ptr(torch.cuda.current_stream(vecs.device)) if on_dev else None
        check(lib.rfx_index_add(self.handle, ptr(vecs), vecs.shape[0], int(on_dev), ctypes.byref(first), st))
        return first.value

    def write(self, row0: int, vecs: torch.Tensor) -> None:
        """Overwrite existing rows [row0, row0 + n) with rows of the index dtype (rfx_index_write): they are
        live again and their int8-copy tiles are re-quantised."""
        if vecs.dim() != 2 or vecs.shape[1] != self.dim or vecs.dtype != self.torch_dtype:
            raise ValueError(f"expected [n][{self.dim}] {self.torch_dtype} rows, got {tuple(vecs.shape)} {vecs.dtype}")
        vecs = vecs.contiguous()
        on_dev = vecs.is_cuda
        st = stream_ptr(torch.cuda.current_stream(vecs.device)) if on_dev else None
        check(lib.rfx_index_write(self.handle, int(row0), ptr(vecs), vecs.shape[0], int(on_dev), st))

    def add_synthetic(self, seed: int, n: int, gen_row0: int = -1, stream=None) -> int:
        """Append n generated rows; generator row ids start at gen_row0 (default: continue)."""
        first = ctypes.c_int64()
        with torch.cuda.device(self.device):
            check(lib.rfx_index_add_synthetic(self.handle, ctypes.c_uint64(seed), int(gen_row0), int(n),
                                              ctypes.byref(first), stream_ptr(stream)))
        return first.value

    def tombstone(self, rows) -> None:
        import numpy as np
        arr = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        with torch.cuda.device(self.device):
            check(lib.rfx_index_tombstone(self.handle, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), arr.size,
                                          stream_ptr()))

    def read(self, row0: int, n: int) -> torch.Tensor:
        out = torch.empty((n, self.dim), dtype=self.torch_dtype, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.rfx_index_read(self.handle, int(row0), int(n), ptr(out), 1, stream_ptr()))
        return out

    # ---- search -------------------------------------------------------------------------------
    def workspace_bytes(self, nq: int, k: int) -> int:
        b = ctypes.c_size_t()
        check(lib.rfx_search_workspace_bytes(self.handle, int(nq), int(k), ctypes.byref(b)))
        return b.value

    def _check_queries(self, q: torch.Tensor):
        if q.dim() != 2 or q.shape[1] != self.dim or q.dtype != self.torch_dtype or not q.is_cuda:
            raise ValueError(f"queries must be a cuda {self.torch_dtype} tensor [nq][{self.dim}]")
        return q.contiguous()

    def _check_mask(self, row_mask, dev):
        """row_mask: None, or a device int32/uint32 bitmap (bit r & 31 of word r >> 5 = row r allowed)
        of at least (rows + 31) // 32 words (make_row_mask)."""
        if row_mask is None:
            return None, 0
        if row_mask.dtype not in (torch.int32, torch.uint32) or row_mask.dim() != 1 or not row_mask.is_contiguous():
            raise ValueError("row mask must be a contiguous 1-D int32/uint32 tensor")
        if row_mask.device != dev:
            raise ValueError(f"row mask on {row_mask.device}, queries on {dev}")
        if row_mask.numel() < (self.rows + 31) // 32:
            raise ValueError(f"row mask has {row_mask.numel()} words, index needs {(self.rows + 31) // 32}")
        return row_mask, row_mask.numel()

    def search(self, queries: torch.Tensor, k: int, workspace: torch.Tensor = None, stream=None,
               row_mask: torch.Tensor = None):
        """Top-k rows per query: (scores f32 [nq][k], rows int64 [nq][k]) on the device.
        row_mask (optional): only rows whose bit is set are returned (metadata filter)."""
        q = self._check_queries(queries)
        nq = q.shape[0]
        dev = q.device
        out_s = torch.empty((nq, k), dtype=torch.float32, device=dev)
        out_r = torch.empty((nq, k), dtype=torch.int64, device=dev)
        need = self.workspace_bytes(nq, k)
        ws = workspace if workspace is not None and workspace.numel() >= need else \
            torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        m, mw = self._check_mask(row_mask, dev)
        with torch.cuda.device(dev):
            if m is None:
                check(lib.rfx_search(self.handle, ptr(q), nq, int(k), ptr(out_s), ptr(out_r), ptr(ws), ws.numel(),
                                     stream_ptr(stream)))
            else:
                check(lib.rfx_search_masked(self.handle, ptr(q), nq, int(k), ptr(m), mw, ptr(out_s), ptr(out_r),
                                            ptr(ws), ws.numel(), stream_ptr(stream)))
        return out_s, out_r

    def search_records(self, queries: torch.Tensor, k: int, row_offset: int = 0, out: torch.Tensor = None,
                       workspace: torch.Tensor = None, stream=None, row_mask: torch.Tensor = None) -> torch.Tensor:
        """The search as [nq][k][2] int64 merge records (score bits, row + row_offset): one shard's
        all-gather input (rfx_search_records; the two-pass scan included)."""
        q = self._check_queries(queries)
        nq = q.shape[0]
        if out is None:
            out = torch.empty((nq, k, 2), dtype=torch.int64, device=q.device)
        elif out.shape != (nq, k, 2) or out.dtype != torch.int64 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous int64 [{nq}][{k}][2] tensor")
        need = self.workspace_bytes(nq, k)
        ws = workspace if workspace is not None and workspace.numel() >= need else \
            torch.empty(max(need, 1), dtype=torch.uint8, device=q.device)
        m, mw = self._check_mask(row_mask, q.device)
        with torch.cuda.device(q.device):
            check(lib.rfx_search_records(self.handle, ptr(q), nq, int(k), ptr(m) if m is not None else None, mw,
                                         int(row_offset), ptr(out), ptr(ws), ws.numel(), stream_ptr(stream)))
        return out

    # ---- the exact two-pass scan (int8 copy of the store) --------------------------------
    def enable_screen(self, mode: int = 1, stream=None) -> None:
        """Keep an int8 copy of the rows (dim bytes per row) and answer searches with the exact
        two-pass scan where it applies (kernel 10: bf16/f16 batches of > 64 questions; kernel 11: up
        to 8 questions of any dtype): int8 screen, exact re-score of the survivors, the exact scan as
        a gated fallback.  mode 0 drops the copy; mode 2 forces the fallback (tests)."""
        with torch.cuda.device(self.device):
            check(lib.rfx_index_screen(self.handle, int(mode), stream_ptr(stream)))

    def screen_state(self):
        """(mode, device bytes of the int8 copy, dropped): dropped = an append outgrew the room the copy
        had (RFX_ECAPACITY) and the library went back to the exact scan."""
        m, b, d = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int()
        check(lib.rfx_index_screen_state(self.handle, ctypes.byref(m), ctypes.byref(b), ctypes.byref(d)))
        return m.value, b.value, bool(d.value)

    def search_plan(self, nq: int, k: int) -> int:
        """Kernel rfx_search runs for (nq, k): 10 = the two-pass scan of a batch (int8 MFMA screen),
        11 = the two-pass scan of up to 8 questions (int8 dot4 screen, one launch)."""
        kern = ctypes.c_int()
        check(lib.rfx_search_plan(self.handle, int(nq), int(k), ctypes.byref(kern)))
        return kern.value

    def screen_read(self, tile0: int, ntiles: int):
        """(codes int8 [ntiles*32][dim], scales f32 [ntiles], live u32 [ntiles], stats f32 [3]: max row norm,
        max quantisation-error norm, max tile scale) of the copy."""
        import numpy as np
        codes = np.empty((ntiles * 32, self.dim), dtype=np.int8)
        scales = np.empty(ntiles, dtype=np.float32)
        live = np.empty(ntiles, dtype=np.uint32)
        stats = np.empty(3, dtype=np.float32)
        with torch.cuda.device(self.device):
            check(lib.rfx_index_screen_read(self.handle, int(tile0), int(ntiles), codes.ctypes.data, scales.ctypes.data,
                                            live.ctypes.data, stats.ctypes.data))
        return codes, scales, live, stats

    def screen_diag(self, nq: int, k: int, workspace: torch.Tensor):
        """After a two-pass search on `workspace`: (diag int32 [nq][2] = kept candidates, survivors
        re-scored (-1: query sent to the fallback); fallback ran for the batch)."""
        import numpy as np
        diag = np.empty((nq, 2), dtype=np.int32)
        fb = ctypes.c_uint32()
        with torch.cuda.device(self.device):
            check(lib.rfx_screen_diag(self.handle, int(nq), int(k), ptr(workspace), diag.ctypes.data, ctypes.byref(fb)))
        return diag, bool(fb.value)

    def list_len(self, nq: int, k: int) -> int:
        """Length of the sorted candidate lists rfx_scan_topk writes (merge hint)."""
        n = ctypes.c_int()
        check(lib.rfx_scan_list_len(self.handle, int(nq), int(k), ctypes.byref(n)))
        return n.value

    def plan(self, nq: int, k: int):
        kern, ncand = ctypes.c_int(), ctypes.c_int64()
        check(lib.rfx_scan_plan(self.handle, int(nq), int(k), ctypes.byref(kern), ctypes.byref(ncand)))
        return kern.value, ncand.value

    def scan(self, queries: torch.Tensor, k: int, workspace: torch.Tensor = None, stream=None,
             row_mask: torch.Tensor = None):
        """Fused scan only: per-query candidate lists (scores f32 [nq][n_cand], local rows int32)."""
        q = self._check_queries(queries)
        nq = q.shape[0]
        _, ncand = self.plan(nq, k)
        cs = torch.empty((nq, ncand), dtype=torch.float32, device=q.device)
        cr = torch.empty((nq, ncand), dtype=torch.int32, device=q.device)
        need = self.workspace_bytes(nq, k)
        ws = workspace if workspace is not None and workspace.numel() >= need else \
            torch.empty(max(need, 1), dtype=torch.uint8, device=q.device)
        m, mw = self._check_mask(row_mask, q.device)
        with torch.cuda.device(q.device):
            if m is None:
                check(lib.rfx_scan_topk(self.handle, ptr(q), nq, int(k), ptr(cs), ptr(cr), ptr(ws), ws.numel(),
                                        stream_ptr(stream)))
            else:
                check(lib.rfx_scan_topk_masked(self.handle, ptr(q), nq, int(k), ptr(m), mw, ptr(cs), ptr(cr),
                                               ptr(ws), ws.numel(), stream_ptr(stream)))
        return cs, cr


def _check_cands(cand_s: torch.Tensor, cand_r: torch.Tensor):
    if cand_s.shape != cand_r.shape or cand_s.dim() != 2:
        raise ValueError("candidate score/row tensors must be [nq][n_cand] of equal shape")
    if cand_r.dtype not in (torch.int32, torch.int64) or cand_s.dtype != torch.float32:
        raise ValueError("candidates must be (float32, int32|int64)")
    return cand_s.contiguous(), cand_r.contiguous()


def topk_merge(cand_s: torch.Tensor, cand_r: torch.Tensor, k: int, row_offset: int = 0, stream=None,
               list_len: int = 1, sorted: bool = False):
    """Merge [nq][n_cand] candidates (rows int32 or int64) into the final top-k per query.
    list_len: the candidates are lists of that length (DeviceIndex.list_len); 1 = no hint.
    sorted: the lists are sorted best first with empty slots at the tail, as DeviceIndex.scan
    writes them (rfx_topk_merge_sorted: a list is read only while it can still contribute)."""
    cand_s, cand_r = _check_cands(cand_s, cand_r)
    nq, ncand = cand_s.shape
    out_s = torch.empty((nq, k), dtype=torch.float32, device=cand_s.device)
    out_r = torch.empty((nq, k), dtype=torch.int64, device=cand_s.device)
    with torch.cuda.device(cand_s.device):
        if sorted:
            check(lib.rfx_topk_merge_sorted(ptr(cand_s), ptr(cand_r), int(cand_r.dtype == torch.int64), nq, ncand,
                                            int(list_len), int(k), int(row_offset), ptr(out_s), ptr(out_r), None,
                                            stream_ptr(stream)))
            return out_s, out_r
        check(lib.rfx_topk_merge_lists(ptr(cand_s), ptr(cand_r), int(cand_r.dtype == torch.int64), nq, ncand,
                                       int(list_len), int(k), int(row_offset), ptr(out_s), ptr(out_r),
                                       stream_ptr(stream)))
    return out_s, out_r


def topk_merge_records(cand_s: torch.Tensor, cand_r: torch.Tensor, k: int, row_offset: int = 0, stream=None,
                       list_len: int = 1, out: torch.Tensor = None, sorted: bool = False) -> torch.Tensor:
    """Merge as topk_merge, writing [nq][k][2] int64 records (score bits, global row): the
    all-gather input of the multi-GPU step (rfx.dist.pack's layout)."""
    cand_s, cand_r = _check_cands(cand_s, cand_r)
    nq, ncand = cand_s.shape
    if out is None:
        out = torch.empty((nq, k, 2), dtype=torch.int64, device=cand_s.device)
    elif out.shape != (nq, k, 2) or out.dtype != torch.int64 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous int64 [{nq}][{k}][2] tensor")
    with torch.cuda.device(cand_s.device):
        if sorted:
            check(lib.rfx_topk_merge_sorted(ptr(cand_s), ptr(cand_r), int(cand_r.dtype == torch.int64), nq, ncand,
                                            int(list_len), int(k), int(row_offset), None, None, ptr(out),
                                            stream_ptr(stream)))
            return out
        check(lib.rfx_topk_merge_records(ptr(cand_s), ptr(cand_r), int(cand_r.dtype == torch.int64), nq, ncand,
                                         int(list_len), int(k), int(row_offset), ptr(out), stream_ptr(stream)))
    return out


def rescore_topk(index: "DeviceIndex", queries: torch.Tensor, scores: torch.Tensor = None, rows: torch.Tensor = None,
                 records: torch.Tensor = None, row_offset: int = 0, stream=None):
    """The score rule of every search (fl32 of the f64 dot; score desc, row asc) applied in place to an
    answer assembled from scan_topk / topk_merge* (rfx_rescore_topk): (scores, rows) [nq][k], or the
    [nq][k][2] records of topk_merge_records (rows carry row_offset).  Returns what it was given."""
    q = index._check_queries(queries)
    nq = q.shape[0]
    if records is not None:
        if records.shape[0] != nq or records.dim() != 3 or records.dtype != torch.int64 or not records.is_contiguous():
            raise ValueError("records must be a contiguous int64 [nq][k][2] tensor")
        k = records.shape[1]
        with torch.cuda.device(q.device):
            check(lib.rfx_rescore_topk(index.handle, ptr(q), nq, int(k), int(row_offset), None, None, ptr(records),
                                       stream_ptr(stream)))
        return records
    if scores.shape != rows.shape or scores.shape[0] != nq or not (scores.is_contiguous() and rows.is_contiguous()):
        raise ValueError("scores / rows must be contiguous [nq][k] tensors")
    with torch.cuda.device(q.device):
        check(lib.rfx_rescore_topk(index.handle, ptr(q), nq, int(scores.shape[1]), int(row_offset), ptr(scores),
                                   ptr(rows), None, stream_ptr(stream)))
    return scores, rows


def merge_gathered(gathered: torch.Tensor, k: int, stream=None):
    """Final merge of all-gathered records [world][nq][k][2] int64 -> (scores [nq][k], rows [nq][k])."""
    if gathered.dim() != 4 or gathered.shape[3] != 2 or gathered.dtype != torch.int64 or gathered.shape[2] != k:
        raise ValueError("gathered must be int64 [world][nq][k][2]")
    g = gathered.contiguous()
    world, nq = g.shape[0], g.shape[1]
    out_s = torch.empty((nq, k), dtype=torch.float32, device=g.device)
    out_r = torch.empty((nq, k), dtype=torch.int64, device=g.device)
    with torch.cuda.device(g.device):
        check(lib.rfx_merge_gathered(ptr(g), int(world), nq, int(k), ptr(out_s), ptr(out_r), stream_ptr(stream)))
    return out_s, out_r


def synth_rows(seed: int, row0: int, n: int, dim: int, dtype: str, device: int = 0) -> torch.Tensor:
    """Synthetic normalised rows generated on the device (same generator as the index)."""
    out = torch.empty((n, dim), dtype=_lib.TORCH_DTYPES[dtype], device=torch.device("cuda", device))
    with torch.cuda.device(device):
        check(lib.rfx_synth_rows(ctypes.c_uint64(seed), int(row0), int(n), int(dim), _lib.DTYPE_CODES[dtype],
                                 ptr(out), stream_ptr()))
    return out
