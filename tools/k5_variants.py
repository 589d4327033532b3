"""Dev tool (debug library): time the headline scan kernel's MODE ablations on the cfg3 corpus the
way the bench runs it — `--burst` launches back to back per measurement (the chip's power limiter
settles on a clock per workload; single launches after an idle gap read fast), variants
interleaved over rounds (cdna_hip_programming.md §5.4 rule 24).

MODE bits (k_scan_mfma5.h): 1 no top-k epilogue, 2 no MFMA, 8 no corpus stream after the prologue,
131072 16x16x32 MFMA shape, 262144 every other A fragment reused (half the LDS reads; wrong
scores, timing only).  Mode numbers passed to rfx_dbg_scan_variant are 1000 + MODE; 3 = the
production plan; 9 = a plain streaming read of the corpus (HBM ceiling)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RFX_LIB", os.path.join(ROOT, "rag-foundation_amd", "rfx", "librfx_dbg.so"))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--burst", type=int, default=30)
ap.add_argument("--modes", default="3,1000,132072,20000000,1009,20000009,20000001,1003")
ap.add_argument("--warm-seconds", type=float, default=2.0)
ap.add_argument("--no-stream-ref", action="store_true")
a = ap.parse_args()
f = _lib.lib.rfx_dbg_scan_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
f.restype = ctypes.c_int
g = _lib.lib.rfx_dbg_stream_read
g.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
g.restype = ctypes.c_int
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
q = synth_rows(1, 0, a.nq, 768, "bf16")
_, ncand = ix.plan(a.nq, a.k)
cs = torch.empty((a.nq, ncand), dtype=torch.float32, device="cuda")
cr = torch.empty((a.nq, ncand), dtype=torch.int32, device="cuda")
ws = torch.empty(ix.workspace_bytes(a.nq, a.k), dtype=torch.uint8, device="cuda")
scratch = torch.zeros(4, dtype=torch.int32, device="cuda")
st = _lib.stream_ptr()
modes = [int(m) for m in a.modes.split(",")] + ([] if a.no_stream_ref else [9])


def launch(m):
    if m == 9:
        _lib.check(g(ix.handle, _lib.ptr(scratch), st))
    else:
        _lib.check(f(ix.handle, _lib.ptr(q), a.nq, a.k, m, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))


# correctness of the production-shaped variants against the production plan (exact rows)
from rfx.index import topk_merge  # noqa: E402

ref = None
check = {}
for m in [3] + [m for m in modes if m in (1000, 132072, 20000000, 20000070, 20000071, 20000064, 20000256, 20000320, 20000512, 20000016)]:
    launch(m)
    s, r = topk_merge(cs, cr, a.k, list_len=ix.list_len(a.nq, a.k))
    if ref is None:
        ref = (s.clone(), r.clone())
    check[m] = bool(torch.equal(r, ref[1])) and float((s - ref[0]).abs().max()) <= 1e-6

t_end = time.time() + a.warm_seconds
while time.time() < t_end:
    launch(3)
    torch.cuda.synchronize()
res = {m: [] for m in modes}
for rnd in range(a.rounds + 1):
    for m in (modes if rnd % 2 == 0 else modes[::-1]):  # alternate the order: no variant always follows the same one
        launch(m)  # settle into this variant
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.burst):
            launch(m)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            res[m].append(e0.elapsed_time(e1) / a.burst)
    print(f"round {rnd} done", file=sys.stderr, flush=True)
alg = a.rows * 768 * 2
out = {m: {"ms_median": round(sorted(v)[len(v) // 2], 4), "ms_min": round(min(v), 4),
           "GBps": round(alg / (sorted(v)[len(v) // 2] * 1e-3) / 1e9, 1)} for m, v in res.items()}
for m, ok in [(m, ok) for m, ok in check.items() if m in out]:
    out[m]["rows_equal_production"] = ok
print(json.dumps(out))
