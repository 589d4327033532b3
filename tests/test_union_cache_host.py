"""CPU: the union-view cache of rfx.retriever: a view's device copy is
built OUTSIDE the process-wide _STATE_LOCK (which every batcher, embedder and union lookup takes), and an
evicted view that is still in use keeps its bytes counted until its last user releases it.

The view class is a host stand-in (no device copy); the cache logic is the product's."""
import threading

from rfx import retriever as rret
from rfx import union as runion


class _Idx:
    def __init__(self, rows):
        self.rows = rows
        self.capacity = rows


import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _copying_views(monkeypatch):
    # the cache logic is the same for both kinds of view; the copying view's byte counts exercise the budget
    monkeypatch.setenv("RFX_UNION_COPY", "1")


class _Store:
    def __init__(self, name, rows):
        self.name, self.generation, self.version = name, "g0", 1
        self.index = _Idx(rows)
        self.dim, self.dtype, self.device, self._screen_on = 768, "bf16", 0, False


class _Registry:
    def __init__(self):
        self.on_evict = []


def _stand_in(started=None, release=None):
    class View:
        built = []

        def __init__(self, stores):
            self.key = runion.union_key(stores)
            self.nbytes = runion.planned_bytes(stores)
            self.users, self.evicted, self.closed = 0, False, False
            if started is not None:
                started.set()
                assert release.wait(10)
            View.built.append(self)

        def follow(self, stores):
            return False

        def close(self):
            self.closed = True

    return View


def test_union_build_runs_outside_the_state_lock(monkeypatch):
    started, release = threading.Event(), threading.Event()
    monkeypatch.setattr(runion, "UnionView", _stand_in(started, release))
    ret = rret.GpuRetriever(registry=_Registry())
    stores = [_Store("ua", 5000), _Store("ub", 7000)]
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("v", ret._union_view(["ua", "ub"], stores)))
    t.start()
    try:
        assert started.wait(10)
        # the view is being built (its device copy): the process-wide lock is free meanwhile, so other
        # chat threads' batcher / embedder / union lookups go on
        assert rret._STATE_LOCK.acquire(timeout=2)
        rret._STATE_LOCK.release()
    finally:
        release.set()
        t.join(10)
    v = out["v"]
    assert v.users == 1 and rret._UNIONS[(("ua", "ub"), id(ret.registry))] is v
    rret._release_union(v)
    rret._purge_batchers("ua")
    assert v.closed and (("ua", "ub"), id(ret.registry)) not in rret._UNIONS


def test_evicted_view_in_use_stays_counted_until_released(monkeypatch):
    View = _stand_in()
    monkeypatch.setattr(runion, "UnionView", View)
    ret = rret.GpuRetriever(registry=_Registry())
    a = [_Store("ea", 4000), _Store("eb", 4000)]
    b = [_Store("ec", 4000), _Store("ed", 4000)]
    one = runion.planned_bytes(a)
    monkeypatch.setenv("RFX_UNION_MAX_BYTES", str(int(one * 1.5)))  # room for one view
    base = rret._UNION_BYTES[0]
    va = ret._union_view(["ea", "eb"], a)  # pinned by this "search"
    assert rret._UNION_BYTES[0] == base + one
    vb = ret._union_view(["ec", "ed"], b)  # evicts va from the cache: va is still in use
    assert va.evicted and not va.closed
    assert rret._UNION_BYTES[0] == base + 2 * one  # both views' device memory is live
    rret._release_union(va)
    assert va.closed and rret._UNION_BYTES[0] == base + one
    rret._release_union(vb)
    rret._purge_batchers("ec")
    assert vb.closed and rret._UNION_BYTES[0] == base


def test_only_the_least_recently_used_view_makes_room(monkeypatch):
    """evicted views stay counted until they are closed after the lock, so the eviction loop
    tallies what it frees itself; a third view evicts the oldest one only, not the whole cache."""
    View = _stand_in()
    monkeypatch.setattr(runion, "UnionView", View)
    ret = rret.GpuRetriever(registry=_Registry())
    a = [_Store("la", 4000), _Store("lb", 4000)]
    b = [_Store("lc", 4000), _Store("ld", 4000)]
    c = [_Store("le", 4000), _Store("lf", 4000)]
    one = runion.planned_bytes(a)
    monkeypatch.setenv("RFX_UNION_MAX_BYTES", str(int(one * 2.5)))  # room for two views
    base = rret._UNION_BYTES[0]
    views = []
    for names, stores in ((["la", "lb"], a), (["lc", "ld"], b), (["le", "lf"], c)):
        v = ret._union_view(names, stores)
        rret._release_union(v)  # the search is done: unpinned
        views.append(v)
    va, vb, vc = views
    assert va.closed and va.evicted
    assert not vb.closed and not vb.evicted and not vc.closed
    keys = [k[0] for k in rret._UNIONS if k[1] == id(ret.registry)]
    assert keys == [("lc", "ld"), ("le", "lf")]
    assert rret._UNION_BYTES[0] == base + 2 * one
    rret._purge_batchers("lc")
    rret._purge_batchers("le")
    assert vb.closed and vc.closed and rret._UNION_BYTES[0] == base
