"""UnionView — one device index over the rows of several stores, so a question over a list of
stores (the file-search tool's `file_search_store_names`, gemini_rag.py:463-469) is ONE scan launch
and one merge instead of one per store plus a host merge.

Zero copy (round 6, the default): rfx_union_create maps the members' device memory (their rows, and their
int8 copies when every member holds one) back to back into one address range through HIP virtual memory, so
the view IS the members' memory.  Member i owns the view rows [base_i, base_i + capacity_i): its rows, then
its NaN tail.  Appends within a member's capacity and tombstones show through at once; `follow` only copies
the members' tile records again (16 B per 32 rows, the view's own bytes with 256 B of stats) and rebuilds
the view — a new mapping, still no copy — when a member moved its memory (growth past its capacity, a
rebuilt or dropped int8 copy).  RFX_UNION_COPY=1 (or a device without virtual memory) keeps the copying
view below.

The copying view:

Layout: store i owns the union row range [base_i, base_i + region_i); its rows [0, rows_i) sit at
[base_i, base_i + rows_i), the rest of the region is NaN headroom (never returned, like a
tombstone).  Bases and regions are multiples of 32 (a row-mask word never straddles two stores).
Ranking in the view is (score desc, union row asc) = (score desc, store order, row asc): exactly
GpuRetriever's per-store merge rule, and each row's score comes from the same kernels on the same
stored values, so the hits are identical to searching the stores one by one.

Following the members: a member's committed state changes by appends and
tombstones only (the same generation).  `follow` copies just the rows a member appended since the
view last looked into its headroom (rfx_index_write: device to device, the int8 copy's touched tiles
re-quantised) and re-applies its new tombstones (LocalStore.tomb_rows) — O(appended rows), not a
rebuild.  Only a member that outgrows its headroom (max(4,096, rows / 16) rows, so the NaN rows the
scan also streams stay ~6 %), a new generation, or a changed store list rebuilds the view.

Eligible: every member a flat DeviceIndex store (IVF stores answer from their lists, sharded stores
from their shards) on one device with one dim / dtype, and RFX_UNION_MAX_ROWS (default 16M) union
rows; the retriever's view cache is bounded in bytes (RFX_UNION_MAX_BYTES, LRU; rfx.retriever).
"""
import ctypes
import os

import numpy as np
import torch

from . import filters
from ._lib import ESIZE, RFX_EUNSUPPORTED, check, lib
from .index import DeviceIndex

ALIGN = 32


def zero_copy() -> bool:
    return os.environ.get("RFX_UNION_COPY", "0") != "1"


def union_key(stores):
    return tuple((st.name, st.generation, st.version, st.index.rows) for st in stores)


def _region(rows: int) -> int:
    """Union rows reserved for a member of `rows` rows: its rows plus headroom for appends."""
    return -(-(rows + max(4096, rows // 16)) // ALIGN) * ALIGN


def planned_rows(stores) -> int:
    if zero_copy():
        return sum(max(st.index.capacity, 1) for st in stores)
    return sum(_region(st.index.rows) for st in stores)


def members_screened(stores) -> bool:
    """The view keeps an int8 copy (and answers with the two-pass scan) when every member does: each
    member's state as it stands (LocalStore._screen_on follows a copy that growth dropped),
    not the first member's.  Either plan returns the same bits (one score rule, k_scan_valu.h)."""
    return all(getattr(st, "_screen_on", False) is True for st in stores)


def planned_bytes(stores) -> int:
    """Device bytes a view over `stores` would hold of its own: zero copy, the tile records of the int8 copy
    (16 B per 32 rows) and its stats when the members answer with the two-pass scan; copying, the rows and
    the int8 copy (dim bytes per row)."""
    st0 = stores[0]
    n = planned_rows(stores)
    if zero_copy():
        return (n // ALIGN * 16 + 256) if members_screened(stores) else 0
    return n * st0.dim * (ESIZE[st0.dtype] + (1 if members_screened(stores) else 0))


def eligible(stores) -> bool:
    if len(stores) < 2:
        return False
    first = stores[0]
    limit = int(os.environ.get("RFX_UNION_MAX_ROWS", str(16 << 20)))
    for st in stores:
        if type(st.index) is not DeviceIndex or st.ivf is not None:
            return False
        if st.device != first.device or st.dim != first.dim or st.dtype != first.dtype:
            return False
    return 0 < planned_rows(stores) <= limit and any(st.index.rows for st in stores)


class UnionView:
    def __init__(self, stores):
        self.key = union_key(stores)
        self.names = [st.name for st in stores]
        self.gens = [st.generation for st in stores]
        st0 = stores[0]
        self.dim, self.dtype, self.device = st0.dim, st0.dtype, st0.device
        self.screened = members_screened(stores)
        self.bases, self.rows, self.regions, self.tombs = [], [], [], []
        self.rows_copied = 0  # rows this view copied from its members (tests / profiles: O(appended))
        self.users, self.evicted = 0, False  # pins of the retriever's view cache (rfx.retriever)
        self.mapped = zero_copy() and self._map(stores)
        if not self.mapped:
            self._build_copy(stores)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(torch.device("cuda", self.device)).cuda_stream)

    def _map(self, stores) -> bool:
        """The zero-copy view (rfx_union_create); False when the device or a member cannot be mapped."""
        n = len(stores)
        handles = (ctypes.c_uint64 * n)(*[st.index.handle for st in stores])
        bases = (ctypes.c_int64 * n)()
        h = ctypes.c_uint64()
        with torch.cuda.device(torch.device("cuda", self.device)):
            rc = lib.rfx_union_create(handles, n, self._stream(), ctypes.byref(h), bases)
        if rc == RFX_EUNSUPPORTED:
            return False
        check(rc)
        self.index = DeviceIndex(self.dim, self.dtype, self.device, _handle=h.value)
        self.bases = [int(b) for b in bases]
        self.rows = [st.index.rows for st in stores]
        self.regions = [st.index.capacity for st in stores]
        self.tombs = [st.tombs for st in stores]
        self._bases = np.asarray(self.bases, dtype=np.int64)
        total = sum(self.regions)
        self.nbytes = (total // ALIGN * 16 + 256) if self.screened else 0  # the view's own device bytes
        return True

    def _build_copy(self, stores):
        total = planned_rows(stores)
        self.index = DeviceIndex(self.dim, self.dtype, self.device, capacity=max(total, 1))
        dev = torch.device("cuda", self.device)
        base = 0
        try:
            with torch.cuda.device(dev):
                for st in stores:
                    n, reg = st.index.rows, _region(st.index.rows)
                    self.bases.append(base)
                    self.rows.append(n)
                    self.regions.append(reg)
                    self.tombs.append(st.tombs)
                    self._copy(st, 0, n, append=True)
                    self.index.add(torch.full((reg - n, self.dim), float("nan"), dtype=self.index.torch_dtype, device=dev))
                    base += reg
                if self.screened:  # members answer with the two-pass scan: so does the view
                    self.index.enable_screen(1)
        except BaseException:
            self.index.close()
            raise
        self._bases = np.asarray(self.bases, dtype=np.int64)
        # device bytes (fixed: a follow writes into the regions' headroom, the rows never change); kept so
        # the retriever's cache can uncount a view after closing it
        self.nbytes = self.index.rows * self.dim * (ESIZE[self.dtype] + (1 if self.screened else 0))

    def _copy(self, st, r0, r1, append=False, base=0):
        span = 1 << 20
        for a in range(r0, r1, span):
            v = st.index.read(a, min(span, r1 - a))
            if append:
                self.index.add(v)
            else:
                self.index.write(base + a, v)
        self.rows_copied += r1 - r0

    def follow(self, stores) -> bool:
        """Bring the view to the members' committed state in place (callers hold every member's
        lock).  False when it cannot (another store list, a new generation, a member past its
        headroom, a member that shrank): then the caller rebuilds the view."""
        if [st.name for st in stores] != self.names or [st.generation for st in stores] != self.gens:
            return False
        if members_screened(stores) != self.screened:
            return False
        if self.mapped:
            # the rows and codes are the members' memory: their appends and tombstones are already in the
            # view; the tile records (and stats) are copied again.  A member that moved its memory: rebuild
            if [st.index.capacity for st in stores] != self.regions:
                return False
            stale = ctypes.c_int()
            with torch.cuda.device(torch.device("cuda", self.device)):
                check(lib.rfx_union_refresh(self.index.handle, self._stream(), ctypes.byref(stale)))
            if stale.value:
                return False
            self.rows = [st.index.rows for st in stores]
            self.tombs = [st.tombs for st in stores]
            self.key = union_key(stores)
            return True
        for st, n0, reg, t0 in zip(stores, self.rows, self.regions, self.tombs):
            if st.index.rows < n0 or st.index.rows > reg or st.tombs < t0:
                return False
        with torch.cuda.device(torch.device("cuda", self.device)):
            for i, st in enumerate(stores):
                n = st.index.rows
                if n > self.rows[i]:  # the member's appended rows, into its headroom
                    self._copy(st, self.rows[i], n, base=self.bases[i])
                    self.rows[i] = n
                if st.tombs > self.tombs[i]:  # its new tombstones
                    dead = st.tomb_rows(self.tombs[i], st.tombs)
                    if dead.size:
                        self.index.tombstone(dead + self.bases[i])
                    self.tombs[i] = st.tombs
        self.key = union_key(stores)
        return True

    def row_mask(self, stores, metadata_filter):
        """Device mask over the union rows of the members' files matching the filter; None when
        no file of any member matches."""
        ranges = []
        for st, base in zip(stores, self.bases):
            ranges += [(base + a, n) for a, n in st.mask_ranges(metadata_filter)]
        if not ranges:
            return None
        return self.index.mask_tensor(filters.row_mask_words(self.index.rows, ranges))

    def locate(self, rows):
        """Union rows -> (member index, member row) arrays (rows < 0 -> member -1)."""
        rows = np.asarray(rows, dtype=np.int64)
        si = np.searchsorted(self._bases, rows, side="right") - 1
        si = np.where(rows >= 0, si, -1)
        return si, np.where(rows >= 0, rows - self._bases[np.maximum(si, 0)], -1)

    def close(self):
        self.index.close()
