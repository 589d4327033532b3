"""Diagnostic: time the production scan and its ablations on the cfg3 corpus.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).  Dev tool, not product.

Modes: 3 = production plan; 10+M = 256x256 kernel ablation M; 20+M = 256-query-stationary kernel
(k_scan_mfma4.h) with MODE bit flags M (1 no epilogue, 2 no MFMA, 4 contiguous ranges, 8 no corpus
stream, 16 count top-k slow-path entries, 32 τ refresh through L1); 9 = plain
dwordx4 streaming read of the corpus (HBM ceiling)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--modes", default="3,0,1,2")
ap.add_argument("--warm-seconds", type=float, default=2.0)
a = ap.parse_args()
f = _lib.lib.rfx_dbg_scan_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
q = synth_rows(1, 0, a.nq, 768, "bf16")
_, ncand = ix.plan(a.nq, 10)
cs = torch.empty((a.nq, ncand), dtype=torch.float32, device="cuda")
cr = torch.empty((a.nq, ncand), dtype=torch.int32, device="cuda")
ws = torch.empty(ix.workspace_bytes(a.nq, 10), dtype=torch.uint8, device="cuda")
st = _lib.stream_ptr()
g = _lib.lib.rfx_dbg_stream_read
g.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
scratch = torch.zeros(4, dtype=torch.int32, device="cuda")
modes = [int(m) for m in a.modes.split(",")] + [9]


def launch(m):
    if m == 9:
        _lib.check(g(ix.handle, _lib.ptr(scratch), st))
    else:
        if 20 <= m < 1000 and (m - 20) & 16:
            cr.zero_()
        _lib.check(f(ix.handle, _lib.ptr(q), a.nq, 10, m, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))


t_end = time.time() + a.warm_seconds  # steady-state clock before timing (MI355X_MICROARCH.md DVFS item 6)
while time.time() < t_end:
    launch(3)
    torch.cuda.synchronize()
res = {m: [] for m in modes}
slow = {}
for rnd in range(a.rounds + 1):
    for m in modes:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch(m)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            res[m].append(e0.elapsed_time(e1))
        if 20 <= m < 1000 and (m - 20) & 16 and rnd == a.rounds:
            slow[m] = int(cr.flatten()[0])
alg = a.rows * 768 * 2
out = {m: {"ms_median": round(sorted(v)[len(v) // 2], 4), "ms_min": round(min(v), 4),
           "GBps": round(alg / (min(v) * 1e-3) / 1e9, 1)} for m, v in res.items()}
for m, c in slow.items():
    out[m]["slow_path_lane_entries"] = c
print(json.dumps(out))
