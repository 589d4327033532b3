"""UnionView — one device index over the rows of several stores, so a question over a list of
stores (the file-search tool's `file_search_store_names`, gemini_rag.py:463-469) is ONE scan launch
and one merge instead of one per store plus a host merge.

Layout: store i's rows [0, rows_i) sit at union rows [base_i, base_i + rows_i), the bases at
multiples of 32 (a row-mask word never straddles two stores); the gap rows up to the next base are
NaN (never returned, like a tombstone).  The view is a device-to-device copy of the stores' rows,
rebuilt when any member's committed state changes (its key: name, generation, version, rows), so
its results are the stores' committed state at the key.  Ranking in the view is (score desc,
union row asc) = (score desc, store order, row asc): exactly GpuRetriever's per-store merge rule,
and each row's score comes from the same kernels on the same stored values, so the hits are
identical to searching the stores one by one.

Eligible: every member a flat DeviceIndex store (IVF stores answer from their lists, sharded stores
from their shards) on one device with one dim / dtype, and RFX_UNION_MAX_ROWS (default 16M) rows
in all; otherwise the retriever keeps the per-store path.
"""
import os

import numpy as np
import torch

from . import filters
from .index import DeviceIndex

ALIGN = 32


def union_key(stores):
    return tuple((st.name, st.generation, st.version, st.index.rows) for st in stores)


def eligible(stores) -> bool:
    if len(stores) < 2:
        return False
    first = stores[0]
    limit = int(os.environ.get("RFX_UNION_MAX_ROWS", str(16 << 20)))
    total = 0
    for st in stores:
        if type(st.index) is not DeviceIndex or st.ivf is not None:
            return False
        if st.device != first.device or st.dim != first.dim or st.dtype != first.dtype:
            return False
        total += -(-st.index.rows // ALIGN) * ALIGN
    return 0 < total <= limit


class UnionView:
    def __init__(self, stores):
        self.key = union_key(stores)
        self.names = [st.name for st in stores]
        st0 = stores[0]
        self.dim, self.dtype, self.device = st0.dim, st0.dtype, st0.device
        self.bases, self.rows = [], []
        padded = [-(-st.index.rows // ALIGN) * ALIGN for st in stores]
        self.index = DeviceIndex(self.dim, self.dtype, self.device, capacity=max(sum(padded), 1))
        dev = torch.device("cuda", self.device)
        span, base = 1 << 20, 0
        try:
            with torch.cuda.device(dev):
                for st, pad in zip(stores, padded):
                    n = st.index.rows
                    self.bases.append(base)
                    self.rows.append(n)
                    for r0 in range(0, n, span):
                        self.index.add(st.index.read(r0, min(span, n - r0)))
                    if pad > n:
                        nan = torch.full((pad - n, self.dim), float("nan"), dtype=self.index.torch_dtype, device=dev)
                        self.index.add(nan)
                    base += pad
                if getattr(st0, "_screen_on", False):  # members answer with the two-pass scan: so does the view
                    self.index.enable_screen(1)
        except BaseException:
            self.index.close()
            raise
        self._bases = np.asarray(self.bases, dtype=np.int64)

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
