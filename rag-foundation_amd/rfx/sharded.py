"""ShardedIndex — one store's rows split row-wise over several GPUs of ONE process (SURVEY §8e
"single process with ncclCommInitAll", §7 "a single index-server process owning the GPUs"), behind
the same interface LocalStore uses for a DeviceIndex, so LocalGpuRag serves a row-sharded corpus
unchanged (RFX_DEVICES=0,1,...,7; gemini_rag.py:463-469 store -> shards, :721-725 selector).

Layout: shard i holds the contiguous global rows [base_i, base_i + rows_i); the bases are fixed
when the store is first loaded (split evenly, at multiples of 32 rows so a row-mask word never
straddles two shards) and rows appended later go to the last shard; when the last shard grows past
twice the mean of the others the split is redone device to device (_resplit: shard 0 keeps its
rows and appends, every other shard is rebuilt from peer-to-peer copies of the old shards' rows;
nothing is re-read from disk).
IVF stores (RFX_INDEX=ivf, config 5) keep one IVF list set per shard under the store's one coarse
quantiser (ShardedIvf below); a search is bit-identical to the same store on one device.
A search: the batch's queries go to every shard's device, each shard runs its whole search into
[nq][k] records with its base added (rfx_search_records: the exact two-pass scan when the shards hold
their int8 copies), one RCCL gather to device 0 over the process's devices
(rfx_gather_records on an ncclCommInitAll group), one rfx_merge_gathered.
Several shards on one device (RFX_DEVICES=0,0,0,0: logical shards, tests) skip the collective:
their records are stacked on that device and merged by the same kernel.
"""
import ctypes
import os
import threading

import numpy as np
import torch

from ._lib import RFX_EINVAL, RfxCapacityError, check, lib
from .dist import RcclComm
from .index import DeviceIndex, merge_gathered, topk_merge_records

ALIGN = 32  # rows per row-mask word


def parse_devices(spec: str):
    """"0,1,2,3" -> [0, 1, 2, 3]; "0x4" -> [0, 0, 0, 0] (logical shards on one device)."""
    spec = spec.strip()
    if "x" in spec:
        d, n = spec.split("x")
        return [int(d)] * int(n)
    return [int(x) for x in spec.split(",") if x.strip()]


class ShardedIndex:
    supports_ivf = True  # IVF stores: ShardedIvf (new_ivf), one list set per shard

    def __init__(self, dim, dtype, devices):
        if not devices:
            raise ValueError("need at least one device")
        self.dim, self.dtype = int(dim), dtype
        self.devices = [int(d) for d in devices]
        self.device = self.devices[0]  # where results (and the embedder's queries) live
        self.shards = [DeviceIndex(self.dim, dtype, d) for d in self.devices]
        self.bases = [0] * len(self.shards)
        self._split = False
        self.generation = 0  # bumped whenever the shard layout changes (ShardedIvf rebuilds its lists)
        self._screen = 0     # the two-pass scan's int8 copies (enable_screen), re-made on new shards
        self.screen_dropped = False  # a shard's copy was dropped by growth: every shard went exact
        self._tombs = []  # tombstoned global rows (re-applied after a re-split)
        distinct = len(set(self.devices)) == len(self.devices)
        self.comm = RcclComm.for_devices(self.devices) if distinct and len(self.devices) > 1 else None
        self._streams = [torch.cuda.Stream(device=d) for d in self.devices]
        # held across a search's enqueue and across re-splits / close: a batch never searches shards
        # another thread is replacing, and two batches never interleave their scans and all-gather
        self._lock = threading.RLock()
        # a search is ONE C-ABI call (rfx_sharded_search) over buffers kept here, grown to the largest batch
        # (RFX_SHARDED_C=0: the per-shard Python path, kept for A/B of the host cost)
        self.c_path = os.environ.get("RFX_SHARDED_C", "1") != "0"
        self._bufs = None

    # ---- shape ---------------------------------------------------------------------------------
    @property
    def rows(self) -> int:
        return self.bases[-1] + self.shards[-1].rows if self._split else sum(s.rows for s in self.shards)

    @property
    def live_rows(self) -> int:
        return sum(s.live_rows for s in self.shards)

    def _locate(self, rows):
        rows = np.asarray(rows, dtype=np.int64)
        sid = np.searchsorted(np.asarray(self.bases), rows, side="right") - 1
        return sid, rows - np.asarray(self.bases)[sid]

    # ---- loads / writes --------------------------------------------------------------------------
    def _cuts(self, upto):
        n = len(self.shards)
        # every base a multiple of ALIGN, also when upto itself is not (a reader opening a store after
        # a small first upload): mask_tensor slices whole mask words per shard
        top = (upto // ALIGN) * ALIGN
        return [min(top, -(-(i * upto // n) // ALIGN) * ALIGN) for i in range(n)] + [upto]

    def _do_split(self, upto):
        cuts = self._cuts(upto)
        for i in range(len(self.shards)):
            self.bases[i] = cuts[i]
        self._split = True
        self.generation += 1
        return cuts

    def rows_sync(self, path: str, upto: int) -> None:
        """Load file rows [rows, upto): the first load splits them over the shards, later ones go
        to the last shard (the store grew)."""
        with self._lock:
            self._rows_sync(path, upto)

    def _rows_sync(self, path: str, upto: int) -> None:
        if not self._split:
            cuts = self._do_split(upto)
            for i, sh in enumerate(self.shards):
                sh.rows_sync(path, cuts[i + 1] - cuts[i], file_base=cuts[i])
            return
        last = self.shards[-1]
        last.rows_sync(path, upto - self.bases[-1], file_base=self.bases[-1])
        self._screen_follow()
        others = [s.rows for s in self.shards[:-1]]
        if others and last.rows > 2 * max(1.0, sum(others) / len(others)) and upto >= 64 * ALIGN * len(self.shards):
            self._resplit(path, upto)

    def _resplit(self, path, upto):
        """Rebalance device to device (ADVICE/VERDICT r2: no reload from disk).  The new cuts only
        move forward (the store grew), so shard 0 keeps its rows and appends its new tail; shard
        i > 0 is rebuilt from peer copies of the old shards' rows [cut_i, cut_i+1) in 1M-row pieces.
        The new shards are complete before the old ones are closed (callers hold self._lock)."""
        old, old_bases = self.shards, list(self.bases)
        cuts = self._cuts(upto)
        span = 1 << 20

        def copy_into(dst, lo, hi):
            for j, (sh, b) in enumerate(zip(old, old_bases)):
                a, e = max(lo, b), min(hi, b + sh.rows)
                for r0 in range(a, e, span):
                    n = min(span, e - r0)
                    dst.add(sh.read(r0 - b, n).to(torch.device("cuda", dst.device)))

        new = [old[0]]
        try:
            copy_into(old[0], old_bases[0] + old[0].rows, cuts[1])
            for i in range(1, len(old)):
                sh = DeviceIndex(self.dim, self.dtype, self.devices[i], capacity=max(cuts[i + 1] - cuts[i], 1))
                new.append(sh)
                copy_into(sh, cuts[i], cuts[i + 1])
        except BaseException:
            for sh in new[1:]:
                sh.close()
            raise
        for sh in old[1:]:
            sh.close()
        self.shards = new
        for i in range(len(new)):
            self.bases[i] = cuts[i]
        self.generation += 1
        if self._tombs:  # a copied tombstoned row is a NaN row: mark it dead in its new shard too
            self._tombstone(np.concatenate(self._tombs))
        if self._screen:
            try:
                for sh in new[1:]:
                    sh.enable_screen(self._screen)
            except RfxCapacityError:  # the re-split shards do not fit their copies: exact on every shard
                for sh in new:
                    sh.enable_screen(0)
                self._screen = 0
                self.screen_dropped = True
            self._screen_follow()  # (shard 0 appended its new tail: its copy may have been dropped)

    def add(self, vecs: torch.Tensor) -> int:
        """Append rows (writer path): they extend the last shard."""
        with self._lock:
            first = self.rows
            self._split = True
            last = self.shards[-1]
            last.add(vecs.to(torch.device("cuda", self.devices[-1])))
            self._screen_follow()
            return first

    def _screen_follow(self) -> None:
        """All or nothing after growth: only the last shard takes appends, and librfx drops
        a shard's int8 copy when an append outgrows the room the copy has (rfx_index_screen_state reports
        it).  Then every shard drops its copy, so every shard answers with the exact plan (the same score
        rule either way, but one plan per store)."""
        if not self._screen:
            return
        if any(sh.screen_state()[0] == 0 for sh in self.shards):
            for sh in self.shards:
                sh.enable_screen(0)
            self._screen = 0
            self.screen_dropped = True

    def screen_state(self):
        """(mode, device bytes of the shards' int8 copies, dropped) — DeviceIndex.screen_state over the
        shards: mode is the store's (0 once any shard lost its copy), dropped = a copy was dropped by
        growth since enable_screen."""
        states = [sh.screen_state() for sh in self.shards]
        mode = self._screen if all(m for m, _, _ in states) else 0
        return mode, sum(b for _, b, _ in states), bool(self.screen_dropped or any(d for _, _, d in states))

    def rows_append(self, path: str, row0: int) -> None:
        """Write global rows [row0, rows) to the row file, shard by shard in row order."""
        for sh, base in zip(self.shards, self.bases):
            if base + sh.rows > row0:
                sh.rows_append(path, max(row0 - base, 0), file_base=base)

    def _tombstone(self, rows):
        sid, local = self._locate(rows)
        for i, sh in enumerate(self.shards):
            sel = local[sid == i]
            if sel.size:
                sh.tombstone(sel)

    def tombstone(self, rows) -> None:
        rows = np.asarray(rows, dtype=np.int64)
        with self._lock:
            self._tombs.append(rows)
            self._tombstone(rows)

    def read(self, row0: int, n: int) -> torch.Tensor:
        parts = []
        for sh, base in zip(self.shards, self.bases):
            lo, hi = max(row0, base), min(row0 + n, base + sh.rows)
            if hi > lo:
                parts.append(sh.read(lo - base, hi - lo).to(torch.device("cuda", self.device)))
        return torch.cat(parts) if parts else torch.empty((0, self.dim), device=torch.device("cuda", self.device))

    def mask_tensor(self, words):
        """Per-shard device slices of a global row mask (shard bases are multiples of 32)."""
        return [torch.from_numpy(np.ascontiguousarray(words[base // ALIGN:])).to(torch.device("cuda", d))
                for base, d in zip(self.bases, self.devices)]

    def close(self) -> None:
        with self._lock:
            self._close()

    def _close(self) -> None:
        for sh in self.shards:
            sh.close()
        if self.comm is not None:
            self.comm.close()
            self.comm = None

    # ---- search --------------------------------------------------------------------------------
    def search(self, queries: torch.Tensor, k: int, row_mask=None):
        with self._lock:
            return self._search(queries, k, row_mask)

    def _search(self, queries: torch.Tensor, k: int, row_mask=None):
        if self.c_path and queries.shape[0] > 0:
            return self._search_c(queries, k, row_mask)
        return self._search_py(queries, k, row_mask)

    def _buffers(self, nq, k, q_dev, exact=False):
        """Per-shard workspaces, records, query copies and the gathered records, kept across searches and
        grown to the largest batch seen; views of them for this batch.  The workspaces are sized once per
        (layout generation, largest batch) with a quarter of headroom; a shard that outgrew its workspace
        makes rfx_sharded_search fail with RFX_EINVAL, and the caller regrows them exactly (exact=True)."""
        n = len(self.shards)
        shared = self.comm is None
        rec_n = nq * k * 2
        b = self._bufs
        if exact or b is None or b["gen"] != self.generation or b["rec_n"] < rec_n or b["q_n"] < nq * self.dim:
            keep = b is not None and b["gen"] == self.generation
            rec_n_a = max(b["rec_n"], rec_n) if keep else rec_n
            q_n_a = max(b["q_n"], nq * self.dim) if keep else nq * self.dim
            nq_a, k_a = (max(b["nq"], nq), max(b["k"], k)) if keep else (nq, k)
            # the workspace a plan needs is not monotone in nq or k (kernel 11's region exists for nq <= 8 only,
            # the VALU and MFMA plans size their lists differently): room for the largest batch seen AND for this
            # one
            ws = [torch.empty(max(sh.workspace_bytes(nq_a, k_a), sh.workspace_bytes(nq, k)) * 5 // 4 + 4096,
                              dtype=torch.uint8, device=torch.device("cuda", d))
                  for sh, d in zip(self.shards, self.devices)]
            dev0 = torch.device("cuda", self.devices[0])
            gathered = torch.empty(n * rec_n_a, dtype=torch.int64, device=dev0)
            recs = None if shared else [torch.empty(rec_n_a, dtype=torch.int64, device=torch.device("cuda", d))
                                        for d in self.devices]
            qb = [None if d == self.devices[0] else
                  torch.empty(q_n_a, dtype=self.shards[i].torch_dtype, device=torch.device("cuda", d))
                  for i, d in enumerate(self.devices)]
            b = self._bufs = {"gen": self.generation, "rec_n": rec_n_a, "q_n": q_n_a, "nq": nq_a, "k": k_a, "ws": ws,
                              "gathered": gathered, "recs": recs, "qb": qb}
        g = b["gathered"][:n * rec_n].view(n, nq, k, 2)
        recs = [g[i] for i in range(n)] if shared else [r[:rec_n] for r in b["recs"]]
        qb = [None if x is None or q_dev.index == d else x[:nq * self.dim]
              for x, d in zip(b["qb"], self.devices)]
        return b["ws"], recs, g, qb

    def _search_c(self, queries: torch.Tensor, k: int, row_mask=None):
        """One rfx_sharded_search call: every shard's search, the exchange and the merge enqueued from C++
        (the per-shard Python path issued each shard's copy, search and exchange itself)."""
        n, nq = len(self.shards), queries.shape[0]
        # the C side reads nq rows of the index dtype and dim from this pointer: the same checks as the
        # per-shard path's search_records, so a wrong dtype or dim raises instead of reading garbage
        q = self.shards[0]._check_queries(queries)
        if q.device.index != self.devices[0]:
            q = q.to(torch.device("cuda", self.devices[0]))
        src = torch.cuda.current_stream(q.device)
        out_s = torch.empty((nq, k), dtype=torch.float32, device=q.device)
        out_r = torch.empty((nq, k), dtype=torch.int64, device=q.device)
        P = ctypes.c_void_p
        handles = (ctypes.c_uint64 * n)(*[sh.handle for sh in self.shards])
        bases = (ctypes.c_int64 * n)(*self.bases)
        streams = (P * n)(*[P(st.cuda_stream) for st in self._streams])
        masks = words = None
        if row_mask is not None:
            masks = (P * n)(*[P(m.data_ptr()) for m in row_mask])
            words = (ctypes.c_int64 * n)(*[m.numel() for m in row_mask])
        comm = self.comm.handle if self.comm is not None else 0
        for attempt in (0, 1):
            ws, recs, gathered, qb = self._buffers(nq, k, q.device, exact=attempt == 1)
            rc = lib.rfx_sharded_search(n, handles, bases, P(q.data_ptr()),
                                        (P * n)(*[P(x.data_ptr()) if x is not None else None for x in qb]), nq, int(k),
                                        masks, words, (P * n)(*[P(w.data_ptr()) for w in ws]),
                                        (ctypes.c_size_t * n)(*[w.numel() for w in ws]),
                                        (P * n)(*[P(r.data_ptr()) for r in recs]), P(gathered.data_ptr()), comm,
                                        P(src.cuda_stream), streams, P(out_s.data_ptr()), P(out_r.data_ptr()))
            if rc != RFX_EINVAL or attempt == 1 or b"workspace too small" not in lib.rfx_last_error():
                check(rc)
                break
        return out_s, out_r

    def _search_py(self, queries: torch.Tensor, k: int, row_mask=None):
        nq = queries.shape[0]
        src = torch.cuda.current_stream(queries.device)
        recs = []
        for i, (sh, base, d, st) in enumerate(zip(self.shards, self.bases, self.devices, self._streams)):
            st.wait_stream(src)
            with torch.cuda.device(d), torch.cuda.stream(st):
                if sh.rows == 0:  # an empty shard still joins the exchange: no candidates
                    rec = torch.empty((nq, k, 2), dtype=torch.int64, device=torch.device("cuda", d))
                    rec[..., 0] = torch.tensor(float("-inf")).view(torch.int32).item()
                    rec[..., 1] = -1
                else:
                    # the shard's whole search (rfx_search_records): the two-pass scan when the shard holds
                    # its int8 copy (kernel 10 for batches, kernel 11 for a few questions), the exact
                    # scan + merge otherwise; records carry the global rows (row_offset = base)
                    q = queries.to(torch.device("cuda", d), non_blocking=True)
                    m = row_mask[i] if row_mask is not None else None
                    rec = sh.search_records(q, k, row_offset=base, stream=st, row_mask=m)
            recs.append(rec)
        st0 = self._streams[0]
        s, r = merge_gathered(self._exchange(recs, nq, k)[0], k, stream=st0)
        src.wait_stream(st0)
        return s, r

    def _exchange(self, recs, nq, k, everywhere=False):
        """Per-shard [nq][k][2] records -> the gathered [G][nq][k][2] records: on device 0 (list of
        one), or with everywhere=True on every shard's device (list per shard, ordered on that
        shard's stream).  Distinct devices: one RCCL all-gather; logical shards: a stack on stream 0."""
        st0 = self._streams[0]
        if self.comm is not None:
            if not everywhere:  # the answer is assembled on device 0: one hop (rfx_gather_records)
                o = torch.empty((len(self.devices), nq, k, 2), dtype=torch.int64, device=torch.device("cuda", self.devices[0]))
                o.record_stream(st0)
                self.comm.gather_records(recs, [o] + [None] * (len(self.devices) - 1), self._streams, root=0)
                return [o]
            outs = []
            for d, st in zip(self.devices, self._streams):
                o = torch.empty((len(self.devices), nq, k, 2), dtype=torch.int64, device=torch.device("cuda", d))
                o.record_stream(st)
                outs.append(o)
            self.comm.allgather_records(recs, outs, self._streams)
            return outs
        for st in self._streams[1:]:
            st0.wait_stream(st)
        with torch.cuda.stream(st0):
            gathered = torch.stack(recs)
        for rec in recs:
            rec.record_stream(st0)
        if not everywhere:
            return [gathered]
        for st in self._streams[1:]:  # logical shards share device 0: the same tensor, after stream 0
            st.wait_stream(st0)
            gathered.record_stream(st)
        return [gathered] * len(self.shards)

    def enable_screen(self, mode: int = 1) -> None:
        """The exact two-pass scan on every shard (DeviceIndex.enable_screen; kept by re-splits): every
        shard keeps its int8 copy and _search runs each shard through rfx_search_records, whose plan is
        the two-pass scan (search_plan 10 / 11) wherever it applies."""
        with self._lock:
            try:
                for sh in self.shards:
                    sh.enable_screen(mode)
            except BaseException:
                # all or nothing (a shard that does not fit its copy: RfxCapacityError): every shard
                # back to the exact scan, then the caller sees the error (rfx.store logs it)
                for sh in self.shards:
                    sh.enable_screen(0)
                self._screen = 0
                raise
            self._screen = int(mode)
            if mode:
                self.screen_dropped = False

    # ---- IVF (config 5) --------------------------------------------------------------------------
    def new_ivf(self, nlist):
        """The IVF index of an RFX_INDEX=ivf store over these shards (rfx.store._new_ivf)."""
        return ShardedIvf(self, nlist)


class ShardedIvf:
    """IVF-Flat int8 over a ShardedIndex (SURVEY §8 config 5 behind the drop-in adapter;
    gemini_rag.py:463-469): one coarse quantiser (the store's committed centroids, loaded on every
    shard's device), each shard holding its rows' part of every posting list.  The interface is
    rfx.ivf.IvfIndex's as rfx.store uses it (train_from, centroid_bytes, load_centroids, add_from,
    rows, search_index, close).

    A search is bit-identical to rfx_ivf_search_rerank on one device holding all rows:
      1. every shard: its rerank_k best rows by int8 score (rfx_ivf_search; score desc, row asc),
         as records with the shard's base added;
      2. exchange + merge of those records = the store's global rerank_k best (the union of the
         per-shard lists contains them, and the ranking rule is the same), on every shard's device;
      3. every shard re-scores the global candidates it owns against its rows (rfx_rerank_candidates:
         the one-device re-rank kernel), keeps its top k as records;
      4. exchange + merge = the top k of the re-scored global candidates.
    Two exchanges of nq * k_ * 16 B per shard (k_ = rerank_k, then k)."""

    def __init__(self, sidx, nlist):
        self.sidx, self.nlist, self.dim = sidx, int(nlist), sidx.dim
        self.device = sidx.device
        self.parts, self._gen, self._raw = [], None, None

    def _fresh_parts(self):
        from .ivf import IvfIndex
        for p in self.parts:
            p.close()
        self.parts = [IvfIndex(self.dim, self.nlist, d) for d in self.sidx.devices]
        if self._raw is not None:
            for p in self.parts:
                p.load_centroids(self._raw)
        self._gen = self.sidx.generation

    @property
    def rows(self) -> int:
        """Rows in the lists; -1 while the shard layout changed since they were built (not ready)."""
        if self._gen != self.sidx.generation or len(self.parts) != len(self.sidx.shards):
            return -1
        return sum(p.rows for p in self.parts)

    def train_from(self, index, row_ids, iters: int = 10) -> None:
        from .ivf import IvfIndex
        t = IvfIndex(self.dim, self.nlist, self.device)
        try:
            t.train_from(index, row_ids, iters)  # index.read: global rows, gathered onto device 0
            self._raw = t.centroid_bytes()
        finally:
            t.close()
        self._fresh_parts()

    def centroid_bytes(self) -> bytes:
        if self._raw is None:
            raise ValueError("untrained")
        return self._raw

    def load_centroids(self, raw: bytes) -> None:
        self._raw = bytes(raw)
        self._fresh_parts()

    def add_from(self, index, upto: int) -> None:
        """Assign every shard's rows not yet in its lists (upto: the store's rows, all on shards)."""
        with self.sidx._lock:
            if self._gen != self.sidx.generation or len(self.parts) != len(self.sidx.shards):
                self._fresh_parts()  # the layout changed: rebuild the lists from the shards' rows
            for p, sh in zip(self.parts, self.sidx.shards):
                p.add_from(sh, sh.rows)

    def search_index(self, queries: torch.Tensor, k: int, nprobe: int, index=None, rerank_k: int = None, stream=None):
        from .ivf import rerank_candidates
        sidx = self.sidx
        rk = max(int(k), 16) if rerank_k is None else int(rerank_k)
        with sidx._lock:
            if self.rows != sidx.rows:
                raise RuntimeError("IVF lists are behind the shards (add_from first)")
            nq = queries.shape[0]
            src = torch.cuda.current_stream(queries.device)
            qs, recs = [], []
            for p, sh, base, d, st in zip(self.parts, sidx.shards, sidx.bases, sidx.devices, sidx._streams):
                st.wait_stream(src)
                with torch.cuda.device(d), torch.cuda.stream(st):
                    q = queries.to(torch.device("cuda", d), non_blocking=True)
                    s, r = p.search(q, rk, nprobe, stream=st)
                    recs.append(topk_merge_records(s, r, rk, row_offset=base, stream=st))
                qs.append(q)
            cands = self._merge_each(sidx._exchange(recs, nq, rk, everywhere=True), rk)
            recs2 = []
            for q, sh, base, d, st, c in zip(qs, sidx.shards, sidx.bases, sidx.devices, sidx._streams, cands):
                with torch.cuda.device(d), torch.cuda.stream(st):
                    rs, rr = rerank_candidates(q, sh.data_ptr(), sh.dtype, base, sh.rows, c, stream=st)
                    recs2.append(topk_merge_records(rs, rr, k, stream=st))
            st0 = sidx._streams[0]
            s, r = merge_gathered(sidx._exchange(recs2, nq, k)[0], k, stream=st0)
            src.wait_stream(st0)
            return s, r

    def _merge_each(self, gathered, k):
        """The global candidate rows on every shard's device (one merge per distinct tensor)."""
        out, memo = [], {}
        for g, st in zip(gathered, self.sidx._streams):
            if id(g) not in memo:
                memo[id(g)] = (merge_gathered(g, k, stream=st)[1], st)
            rows, mst = memo[id(g)]
            if mst is not st:  # logical shards: the one merge, ordered before this shard's stream
                st.wait_stream(mst)
                rows.record_stream(st)
            out.append(rows)
        return out

    def close(self) -> None:
        for p in self.parts:
            p.close()
        self.parts = []
