"""ShardedIndex — one store's rows split row-wise over several GPUs of ONE process (SURVEY §8e
"single process with ncclCommInitAll", §7 "a single index-server process owning the GPUs"), behind
the same interface LocalStore uses for a DeviceIndex, so LocalGpuRag serves a row-sharded corpus
unchanged (RFX_DEVICES=0,1,...,7; gemini_rag.py:463-469 store -> shards, :721-725 selector).

Layout: shard i holds the contiguous global rows [base_i, base_i + rows_i); the bases are fixed
when the store is first loaded (split evenly, at multiples of 32 rows so a row-mask word never
straddles two shards) and rows appended later go to the last shard; when the last shard grows past
twice the mean of the others the split is redone from the store's row file.
A search: the batch's queries go to every shard's device, each shard runs the fused scan + its
merge into [nq][k] records with its base added (rfx_topk_merge_records), one RCCL all-gather over
the process's devices (rfx_allgather_records on an ncclCommInitAll group), one rfx_merge_gathered.
Several shards on one device (RFX_DEVICES=0,0,0,0: logical shards, tests) skip the collective:
their records are stacked on that device and merged by the same kernel.
"""
import threading

import numpy as np
import torch

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
    supports_ivf = False  # IVF stores keep the exact scan when row-sharded (rfx.store)

    def __init__(self, dim, dtype, devices):
        if not devices:
            raise ValueError("need at least one device")
        self.dim, self.dtype = int(dim), dtype
        self.devices = [int(d) for d in devices]
        self.device = self.devices[0]  # where results (and the embedder's queries) live
        self.shards = [DeviceIndex(self.dim, dtype, d) for d in self.devices]
        self.bases = [0] * len(self.shards)
        self._split = False
        self._tombs = []  # tombstoned global rows (re-applied after a re-split)
        distinct = len(set(self.devices)) == len(self.devices)
        self.comm = RcclComm.for_devices(self.devices) if distinct and len(self.devices) > 1 else None
        self._streams = [torch.cuda.Stream(device=d) for d in self.devices]
        # held across a search's enqueue and across re-splits / close: a batch never searches shards
        # another thread is replacing, and two batches never interleave their scans and all-gather
        self._lock = threading.RLock()

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
    def _do_split(self, upto):
        n = len(self.shards)
        # every base a multiple of ALIGN, also when upto itself is not (a reader opening a store after
        # a small first upload): mask_tensor slices whole mask words per shard
        top = (upto // ALIGN) * ALIGN
        cuts = [min(top, -(-(i * upto // n) // ALIGN) * ALIGN) for i in range(n)] + [upto]
        for i in range(n):
            self.bases[i] = cuts[i]
        self._split = True
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
        others = [s.rows for s in self.shards[:-1]]
        if others and last.rows > 2 * max(1.0, sum(others) / len(others)) and upto >= 64 * ALIGN * len(self.shards):
            self._resplit(path, upto)

    def _resplit(self, path, upto):
        for sh in self.shards:
            sh.close()
        self.shards = [DeviceIndex(self.dim, self.dtype, d) for d in self.devices]
        self._split = False
        self._rows_sync(path, upto)
        if self._tombs:
            self._tombstone(np.concatenate(self._tombs))

    def add(self, vecs: torch.Tensor) -> int:
        """Append rows (writer path): they extend the last shard."""
        with self._lock:
            first = self.rows
            self._split = True
            last = self.shards[-1]
            last.add(vecs.to(torch.device("cuda", self.devices[-1])))
            return first

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
                    q = queries.to(torch.device("cuda", d), non_blocking=True)
                    m = row_mask[i] if row_mask is not None else None
                    cs, cr = sh.scan(q, k, stream=st, row_mask=m)
                    rec = topk_merge_records(cs, cr, k, row_offset=base, stream=st, list_len=sh.list_len(nq, k),
                                             sorted=True)
            recs.append(rec)
        st0 = self._streams[0]
        if self.comm is not None:
            outs = []
            for d, st in zip(self.devices, self._streams):
                o = torch.empty((len(self.devices), nq, k, 2), dtype=torch.int64, device=torch.device("cuda", d))
                o.record_stream(st)
                outs.append(o)
            self.comm.allgather_records(recs, outs, self._streams)
            gathered = outs[0]
        else:
            for st in self._streams[1:]:
                st0.wait_stream(st)
            with torch.cuda.stream(st0):
                gathered = torch.stack(recs)
            for rec in recs:
                rec.record_stream(st0)
        s, r = merge_gathered(gathered, k, stream=st0)
        src.wait_stream(st0)
        return s, r
