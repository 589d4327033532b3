"""Dev tool (debug library): where config 2's time goes.  For several corpus sizes (f32, d 768,
4 rotating copies so no copy is cache-resident), per-launch time of (a) a plain streaming read of
the corpus (the HBM ceiling for that size), (b) the VALU scan alone (rfx_scan_topk), (c) the
one-launch search (rfx_search), measured with HIP events over bursts of back-to-back launches."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RFX_LIB", os.path.join(ROOT, "rag-foundation_amd", "rfx", "librfx_dbg.so"))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", default="25000,50000,100000,200000,400000,1000000")
ap.add_argument("--copies", type=int, default=4)
ap.add_argument("--iters", type=int, default=400)
ap.add_argument("--nq", type=int, default=1)
a = ap.parse_args()
g = _lib.lib.rfx_dbg_stream_read
g.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
g.restype = ctypes.c_int
lib, check, ptr = _lib.lib, _lib.check, _lib.ptr
st = _lib.stream_ptr()
scratch = torch.zeros(4, dtype=torch.int32, device="cuda")
out = {}
for n in [int(x) for x in a.rows.split(",")]:
    ixs = []
    for c in range(a.copies):
        ix = DeviceIndex(768, "f32", 0, capacity=n)
        ix.add_synthetic(c, n)
        ixs.append(ix)
    q = synth_rows(99, 0, a.nq, 768, "f32")
    _, ncand = ixs[0].plan(a.nq, 10)
    cs = torch.empty((a.nq, ncand), dtype=torch.float32, device="cuda")
    cr = torch.empty((a.nq, ncand), dtype=torch.int32, device="cuda")
    os_ = torch.empty((a.nq, 10), dtype=torch.float32, device="cuda")
    or_ = torch.empty((a.nq, 10), dtype=torch.int64, device="cuda")
    ws = torch.empty(ixs[0].workspace_bytes(a.nq, 10), dtype=torch.uint8, device="cuda")

    def run(kind, i):
        h = ixs[i % a.copies].handle
        if kind == "stream":
            check(g(h, ptr(scratch), st))
        elif kind == "scan":
            check(lib.rfx_scan_topk(h, ptr(q), a.nq, 10, ptr(cs), ptr(cr), ptr(ws), ws.numel(), st))
        else:
            check(lib.rfx_search(h, ptr(q), a.nq, 10, ptr(os_), ptr(or_), ptr(ws), ws.numel(), st))

    res = {}
    for kind in ("stream", "scan", "search", "stream", "scan", "search"):
        for i in range(50):
            run(kind, i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            run(kind, i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        res[kind] = min(res.get(kind, 1e9), round(us, 2))
    res["GBps_stream"] = round(n * 768 * 4 / res["stream"] / 1e3, 1)
    res["GBps_scan"] = round(n * 768 * 4 / res["scan"] / 1e3, 1)
    out[n] = res
    print(n, json.dumps(res), flush=True)
    del ixs
    torch.cuda.empty_cache()
