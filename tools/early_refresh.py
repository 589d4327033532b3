"""Dev tool: production scan vs the early-refresh ablation (MODE 4194304) at shard sizes of
1/8, 1/2 and 1x config 3 — time and top-k slow-path entries (MODE | 16 counts into cand_r[0])."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

f = _lib.lib.rfx_dbg_scan_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
out = {}
for rows in (65536, 1_250_000, 2_500_000, 10_000_000):
    ix = DeviceIndex(768, "bf16", 0, capacity=rows)
    ix.add_synthetic(0, rows)
    q = synth_rows(1, 0, 256, 768, "bf16")
    _, ncand = ix.plan(256, 10)
    cs = torch.empty((256, ncand), dtype=torch.float32, device="cuda")
    cr = torch.empty((256, ncand), dtype=torch.int32, device="cuda")
    ws = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
    st = _lib.stream_ptr()

    def run(mode, n=20):
        for _ in range(3):
            _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def slow(mode):
        cr.zero_()
        _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        torch.cuda.synchronize()
        return int(cr.view(-1)[0])

    r = {}
    for rep in range(2):
        for mode in (1000, 1000 + 4194304, 1000 + 8388608):
            r.setdefault(str(mode), []).append(round(run(mode), 4))
    r["slow_prod"] = slow(1000 + 16)
    r["slow_early"] = slow(1000 + 4194320)
    r["slow_early4"] = slow(1000 + 8388624)
    out[rows] = r
    print(rows, json.dumps(r), flush=True)
    del ix
