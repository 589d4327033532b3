"""Dev tool (debug library): where kernel 10's slow path is spent, by tile index (debug MODE 8192: per
tile index of a block's sequence, capped at 63, the wave-tiles that enter the slow path and the
pop-loop trips they make, summed over all waves of `--reps` launches).  The bound's warm-up shows as
the entries and trips of the first tile indices."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RFX_LIB", os.path.join(ROOT, "rag-foundation_amd", "rfx", "librfx_dbg.so"))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_250_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variant", type=int, default=1010493952, help="a MODE-8192 variant (10**8 * RING + MODE; production + 8192 by default)")
a = ap.parse_args()
f = _lib.lib.rfx_dbg_screen_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_size_t, ctypes.c_void_p]
f.restype = ctypes.c_int
g = _lib.lib.rfx_dbg_k10_trips
g.argtypes = [ctypes.c_void_p, ctypes.c_int]
g.restype = ctypes.c_int
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
ix.enable_screen(1)
q = synth_rows(1, 0, 256, 768, "bf16")
ws = torch.empty(ix.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
st = _lib.stream_ptr()
_lib.check(f(ix.handle, _lib.ptr(q), 256, 10, a.variant, _lib.ptr(ws), ws.numel(), st))  # warm
torch.cuda.synchronize()
_lib.check(g(None, 1))
for _ in range(a.reps):
    _lib.check(f(ix.handle, _lib.ptr(q), 256, 10, a.variant, _lib.ptr(ws), ws.numel(), st))
torch.cuda.synchronize()
t = np.zeros((2, 64), dtype=np.uint32)
_lib.check(g(t.ctypes.data, 0))
ent, trips = t[0].astype(np.int64) / a.reps, t[1].astype(np.int64) / a.reps
waves = 256 * 8
print(json.dumps({"rows": a.rows, "waves": waves, "per_wave_by_tile_index": {
    "entries": [round(x / waves, 3) for x in ent[:16]], "trips": [round(x / waves, 3) for x in trips[:16]]},
    "entries_total_per_wave": round(float(ent.sum()) / waves, 2), "trips_total_per_wave": round(float(trips.sum()) / waves, 2),
    "trips_tiles_0_3_per_wave": round(float(trips[:4].sum()) / waves, 2),
    "trips_tiles_0_15_per_wave": round(float(trips[:16].sum()) / waves, 2),
    "note": "index 63 holds every later tile"}, indent=1))
