"""Dev tool: scan_mfma5 time vs rows per block (1..64 tiles of 32 rows per workgroup) for the
production kernel and its stream-only (MODE 3) / MFMA-only (MODE 9) ablations: separates the
per-launch fixed cost from the per-tile cost."""
import ctypes
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
q = synth_rows(1, 0, 256, 768, "bf16")
for tiles in (1, 2, 4, 8, 16, 64):
    rows = 256 * 32 * tiles
    ix = DeviceIndex(768, "bf16", 0, capacity=rows)
    ix.add_synthetic(0, rows)
    _, ncand = ix.plan(256, 10)
    cs = torch.empty((256, ncand), dtype=torch.float32, device="cuda")
    cr = torch.empty((256, ncand), dtype=torch.int32, device="cuda")
    ws = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
    st = _lib.stream_ptr()
    res = []
    for mode in (1000, 1003, 1009):
        for _ in range(5):
            _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        e1.record()
        torch.cuda.synchronize()
        res.append(round(e0.elapsed_time(e1) / 50 * 1e3, 1))
    print(f"tiles/block {tiles:3d} rows {rows:8d}: prod {res[0]} us, stream-only {res[1]} us, mfma-only {res[2]} us",
          flush=True)
    del ix
