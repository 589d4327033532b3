"""GpuRetriever — the index-write / search engine behind LocalGpuRag.

Every call goes to the HIP library (librfx.so); there is no CPU path.
"""
import collections
import os
import threading
from dataclasses import dataclass

import torch

from . import filters
from .batcher import GroupBatcher
from .embedder import DEFAULT_MAX_TOKENS, DEFAULT_OVERLAP, Embedder
from .store import registry as default_registry
from . import union as runion


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


# Process-wide state: get_rag_client() builds a new adapter (and retriever) per request
# (chat.py:937, ingestion.py:214), so embedders and batchers live at module level — one per
# (device, dim) and per store — or no two requests would ever share a batch.
_STATE_LOCK = threading.Lock()
_EMBEDDERS = {}
_BATCHERS = {}  # (store name | tuple of names, filter key, registry id) -> GroupBatcher
# (tuple of names, registry id) -> UnionView (rfx.union), least recently used first; it follows its
# members' appends and tombstones in place.  Bounded in device bytes (RFX_UNION_MAX_BYTES, default
# 32 GiB): the least recently used views are evicted, and a view over its own budget is not built
# (that question takes the per-store path).  A view in use when evicted is closed by its last user.
_UNIONS = collections.OrderedDict()
_UNION_BYTES = [0]


def union_budget() -> int:
    return int(os.environ.get("RFX_UNION_MAX_BYTES", str(32 << 30)))


def _evict_union(key, closing):
    """(caller holds _STATE_LOCK) Drop the view from the cache; an unpinned view goes to `closing`, which the
    caller closes after releasing the lock.  Its bytes stay counted until it is closed (a pinned view's
    device memory lives until its last user releases it: ADVICE r4)."""
    v = _UNIONS.pop(key)
    v.evicted = True
    if v.users == 0:
        closing.append(v)


def _close_unions(closing):
    """Close evicted views outside _STATE_LOCK (hipFree may wait for the device), then uncount them."""
    nbytes = sum(v.nbytes for v in closing)
    for v in closing:
        v.close()
    if closing:
        with _STATE_LOCK:
            _UNION_BYTES[0] -= nbytes


def _release_union(v):
    closing = []
    with _STATE_LOCK:
        v.users -= 1
        if v.evicted and v.users == 0:
            closing.append(v)
    _close_unions(closing)


def _purge_batchers(name):
    closing = []
    with _STATE_LOCK:
        for key in [k for k in _BATCHERS if k[0] == name or (isinstance(k[0], tuple) and name in k[0])]:
            del _BATCHERS[key]
        for key in [k for k in _UNIONS if name in k[0]]:
            _evict_union(key, closing)
    _close_unions(closing)


class GpuRetriever:
    def __init__(self, registry=None, dim=None, dtype=None):
        self._registry = registry
        self.dim = int(os.environ.get("RFX_DIM", "768")) if dim is None else int(dim)
        # bf16 stores by default: half the HBM bytes of f32, and the bf16 MFMA scans run 8x the f32
        # matrix rate.  An f32 store's micro-batches of more than 16 questions run kernel 9 (f32
        # MFMA, one corpus pass per 128 queries); smaller ones the VALU scan in 8-query slices.
        # Parity is defined on the stored values (the oracle widens stored rows exactly), so bf16
        # loses nothing against it; RFX_DTYPE=f32 keeps full-precision vectors where the
        # application wants them.
        self.dtype = os.environ.get("RFX_DTYPE", "bf16") if dtype is None else dtype
        # micro-batching of concurrent questions per store (RFX_BATCH=0 disables)
        self.batching = os.environ.get("RFX_BATCH", "1") != "0"
        # a question over several stores: one scan of their union (rfx.union; RFX_UNION=0 disables)
        self.union = os.environ.get("RFX_UNION", "1") != "0"
        self.last_path = None  # "union" | "per-store" (tests, diagnostics)

    @property
    def registry(self):
        return self._registry or default_registry()

    def embedder(self, dim) -> Embedder:
        key = (self.registry.device, dim)
        with _STATE_LOCK:
            e = _EMBEDDERS.get(key)
            if e is None:
                e = Embedder(dim=dim, device=self.registry.device)
                _EMBEDDERS[key] = e
            return e

    # ---- store namespace ----------------------------------------------------------------------
    def create_store(self, display_name):
        return self.registry.create(display_name, self.dim, self.dtype).name

    def drop_store(self, name):
        _purge_batchers(name)
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
    def _search_store_batch(self, st, items, row_mask=None):
        """One GPU search for a batch of (question, k) against one store: one embedding GEMM,
        one scan + merge at the largest k; each item gets its own first k."""
        kmax = max(k for _, k in items)
        with torch.cuda.device(st.device):
            q = self.embedder(st.dim).embed_texts([t for t, _ in items], st.dtype)
            s, r = st.search(q, kmax, row_mask=row_mask)
            s, r = s.cpu().tolist(), r.cpu().tolist()
        return [(s[i][:k], r[i][:k]) for i, (_, k) in enumerate(items)]

    def _run_batch(self, name, metadata_filter, items):
        """Batch runner: resolves the store and its row mask when the batch runs (a batcher holds
        no LocalStore, so a store that another process replaced or dropped is freed here too)."""
        st = self.registry.get(name)
        if st is None:
            return [None] * len(items)
        mask = st.row_mask(metadata_filter) if metadata_filter is not None else None
        if metadata_filter is not None and mask is None:
            return [None] * len(items)
        return [(st, s, r) for s, r in self._search_store_batch(st, items, mask)]

    def _batcher(self, name, metadata_filter):
        # one batcher per (store, filter): a launch applies one row mask to all its queries
        key = (name, filters.filter_key(metadata_filter), id(self.registry))
        with _STATE_LOCK:
            b = _BATCHERS.get(key)
            if b is None:
                if self.registry.on_evict.count(_purge_batchers) == 0:
                    self.registry.on_evict.append(_purge_batchers)
                b = GroupBatcher(lambda items, n=name, f=metadata_filter: self._run_batch(n, f, items),
                                 max_batch=256)
                if len(_BATCHERS) >= 4096:
                    _BATCHERS.clear()
                _BATCHERS[key] = b
            return b

    def search_store(self, name, question, k, metadata_filter=None):
        """(store, scores, rows) of one question against one store, or None when the store is
        gone or the filter selects no row of it; batched with concurrent callers of the same
        store and filter."""
        if self.batching:
            return self._batcher(name, metadata_filter).submit((question, int(k)))
        return self._run_batch(name, metadata_filter, [(question, int(k))])[0]

    # ---- several stores in one launch (rfx.union) ------------------------------------------------
    def _union_view(self, names, stores):
        """The cached view over `stores` brought up to date (in place when the members only grew or
        deleted rows), pinned for the caller (_release_union), or None when a view of this size does not
        fit the cache's byte budget.  Callers hold every member's lock.

        The device copies (a view's build, a follow's appended rows) run OUTSIDE _STATE_LOCK (VERDICT r4
        #7): that lock guards the cache's dict and counters only, and every batcher, embedder and union
        lookup of the process takes it, so a copy under it would stall every chat thread.  What serialises
        the copies is the member locks the caller holds: every user of a view holds all of its members'
        locks (the key is the member list), so no other thread searches or follows this view meanwhile."""
        key = (tuple(names), id(self.registry))
        want = runion.union_key(stores)
        closing = []
        with _STATE_LOCK:
            v = _UNIONS.get(key)
            if v is not None:
                _UNIONS.move_to_end(key)
                v.users += 1  # pinned: an eviction meanwhile leaves it open for us
        if v is not None:
            ok = v.key == want
            if not ok:
                try:
                    ok = v.follow(stores)
                except BaseException:
                    _release_union(v)
                    raise
            if ok:
                return v
            with _STATE_LOCK:
                if _UNIONS.get(key) is v:
                    _evict_union(key, closing)
            _release_union(v)
        _close_unions(closing)
        closing = []
        need, budget = runion.planned_bytes(stores), union_budget()
        if need > budget:
            return None
        with _STATE_LOCK:  # room for it (bytes reserved while it is built)
            # an evicted view stays counted until _close_unions uncounts it (after the lock), so the loop
            # keeps its own tally of what the evictions free: only the least recently used views that make
            # room go.  A pinned view frees nothing until its last user releases it.
            freed = 0
            while _UNIONS and _UNION_BYTES[0] - freed + need > budget:
                n0 = len(closing)
                _evict_union(next(iter(_UNIONS)), closing)
                freed += sum(v.nbytes for v in closing[n0:])
            _UNION_BYTES[0] += need
            if self.registry.on_evict.count(_purge_batchers) == 0:
                self.registry.on_evict.append(_purge_batchers)
        _close_unions(closing)
        closing = []
        try:
            v = runion.UnionView(stores)
        except BaseException:
            with _STATE_LOCK:
                _UNION_BYTES[0] -= need
            raise
        v.users, v.evicted = 1, False
        with _STATE_LOCK:
            _UNION_BYTES[0] += v.nbytes - need
            if key in _UNIONS:  # (cannot happen while the caller holds the member locks; stay consistent)
                _evict_union(key, closing)
            _UNIONS[key] = v
        _close_unions(closing)
        return v

    def _run_union_batch(self, names, metadata_filter, items):
        """Batch runner over a store list: one embedding GEMM, one scan + merge of the members'
        union.  Returns per item [(score, member index, row, store)] or None per item when the
        list is not eligible (then the caller takes the per-store path)."""
        stores = [self.registry.get(n) for n in names]
        if any(st is None for st in stores) or not runion.eligible(stores):
            return [None] * len(items)
        locked = sorted(set(stores), key=lambda st: st.name)  # one global order: no lock-order deadlock
        for st in locked:  # members hold their locks while the view is built and searched
            st.lock.acquire()
        view = None
        try:
            view = self._union_view(names, stores)
            if view is None:  # over the view cache's byte budget: the per-store path
                return [None] * len(items)
            mask = view.row_mask(stores, metadata_filter) if metadata_filter is not None else None
            if metadata_filter is not None and mask is None:
                return [[] for _ in items]
            kmax = max(k for _, k in items)
            with torch.cuda.device(view.device):
                q = self.embedder(view.dim).embed_texts([t for t, _ in items], view.dtype)
                s, r = view.index.search(q, kmax, row_mask=mask)
                s, r = s.cpu().numpy(), r.cpu().numpy()
            si, lr = view.locate(r)
            out = []
            for i, (_, k) in enumerate(items):
                out.append([(float(s[i, j]), int(si[i, j]), int(lr[i, j]), stores[si[i, j]])
                            for j in range(k) if r[i, j] >= 0])
            return out
        finally:
            if view is not None:
                _release_union(view)
            for st in reversed(locked):
                st.lock.release()

    def _search_union(self, names, question, k, filt):
        if self.batching:
            key = (tuple(names), filters.filter_key(filt), id(self.registry))
            with _STATE_LOCK:
                b = _BATCHERS.get(key)
                if b is None:
                    b = GroupBatcher(lambda items, n=tuple(names), f=filt: self._run_union_batch(n, f, items),
                                     max_batch=256)
                    if len(_BATCHERS) >= 4096:
                        _BATCHERS.clear()
                    _BATCHERS[key] = b
            return b.submit((question, int(k)))
        return self._run_union_batch(tuple(names), filt, [(question, int(k))])[0]

    def search(self, store_names, question, k, metadata_filter=None):
        """Top-k hits over the union of the named stores, rank order (score desc, store order,
        row asc).  metadata_filter: {key: scalar | [scalars]} over upload metadata (rfx.filters).
        Several flat stores on one device: one scan of their union (rfx.union)."""
        k = int(k)
        if not 1 <= k <= 64:
            raise ValueError(f"top_k={k} out of range [1, 64]")
        filt = filters.check_filter(metadata_filter)
        names = list(dict.fromkeys(store_names or []))
        if self.union and len(names) > 1:
            res = self._search_union(names, question, k, filt)
            if res is not None:
                self.last_path = "union"
                hits = []
                for sc, si, row, st in res:
                    info = st.row_info(row)
                    if info is None:
                        continue
                    fid, text, title, uri = info
                    hits.append(Hit(sc, names[si], row, fid, text, title, uri))
                return hits[:k]
        self.last_path = "per-store"
        hits = []
        for si, name in enumerate(names):
            st = self.registry.get(name)
            if st is None or st.index.rows == 0:
                continue
            res = self.search_store(name, question, k, filt)
            if res is None:
                continue
            st, s, r = res
            for sc, row in zip(s, r):
                info = st.row_info(row) if row >= 0 else None
                if info is None:
                    continue
                fid, text, title, uri = info
                hits.append((-sc, si, row, Hit(sc, name, row, fid, text, title, uri)))
        hits.sort(key=lambda h: h[:3])
        return [h[3] for h in hits[:k]]
