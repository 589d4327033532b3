"""Dev tool (debug library): kernel 10's per-block wall clocks (debug MODE 65536: start and end of
every block, 100 MHz) on a synthetic bf16 corpus: how long the slowest block keeps the kernel alive
after the typical one is done (the tail a dynamic tile schedule could remove).
Prints medians over repetitions of: start skew, block duration (median / p90 / max), the end of the
median block and of the last block relative to the first start."""
import argparse
import ctypes
import json
import time
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
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--variant", type=int, default=1010551296,
                help="1010551296 = production (RING 10, per-tile barrier, publish on change) + clocks (10**8 * RING + MODE)")
ap.add_argument("--warm-seconds", type=float, default=3.0, help="back-to-back launches first (the clock under load)")
a = ap.parse_args()
f = _lib.lib.rfx_dbg_screen_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_size_t, ctypes.c_void_p]
f.restype = ctypes.c_int
g = _lib.lib.rfx_dbg_k10_block_times
g.argtypes = [ctypes.c_void_p]
g.restype = ctypes.c_int
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
ix.enable_screen(1)
q = synth_rows(1, 0, a.nq, 768, "bf16")
ws = torch.empty(ix.workspace_bytes(a.nq, a.k), dtype=torch.uint8, device="cuda")
st = _lib.stream_ptr()
ntiles = -(-a.rows // 32)
recs = []
t_end = time.time() + a.warm_seconds
while time.time() < t_end:
    for _ in range(20):
        _lib.check(f(ix.handle, _lib.ptr(q), a.nq, a.k, a.variant, _lib.ptr(ws), ws.numel(), st))
    torch.cuda.synchronize()
for rep in range(a.reps):
    _lib.check(f(ix.handle, _lib.ptr(q), a.nq, a.k, a.variant, _lib.ptr(ws), ws.numel(), st))
    torch.cuda.synchronize()
    bt = np.zeros((1024, 4), dtype=np.uint64)
    _lib.check(g(bt.ctypes.data))
    nb = min(256, ntiles)
    t = bt[:nb, :2].astype(np.int64) * 10  # ns
    ck = bt[:nb, 2:].astype(np.int64)  # shader clock ticks
    clk_mhz = (ck[:, 1] - ck[:, 0]) / np.maximum(t[:, 1] - t[:, 0], 1) * 1e3
    t0 = t[:, 0].min()
    dur = t[:, 1] - t[:, 0]
    ends = t[:, 1] - t0
    xcd = [int(np.median(dur[x::8])) for x in range(8)]  # block b runs on XCD b % 8
    recs.append({"xcd_dur_med_ns": xcd, "slowest_blocks": [int(b) for b in np.argsort(-dur)[:8]],
                 "start_skew_ns": int(t[:, 0].max() - t0), "dur_med_ns": int(np.median(dur)),
                 "dur_p90_ns": int(np.percentile(dur, 90)), "dur_max_ns": int(dur.max()),
                 "end_med_ns": int(np.median(ends)), "end_max_ns": int(ends.max()),
                 "tail_ns": int(ends.max() - np.median(ends)), "clock_mhz_med": int(np.median(clk_mhz))})
keys = [k for k in recs[0] if k not in ("xcd_dur_med_ns", "slowest_blocks")]
med = {k: int(np.median([r[k] for r in recs[a.reps // 4:]])) for k in keys}
med["xcd_dur_med_ns"] = [int(x) for x in np.median([r["xcd_dur_med_ns"] for r in recs[a.reps // 4:]], axis=0)]
med["slowest_blocks_last_rep"] = recs[-1]["slowest_blocks"]
med["slowest_blocks_first_rep"] = recs[a.reps // 4]["slowest_blocks"]
tiles = [(ntiles - b + 255) // 256 for b in range(min(256, ntiles))]
med["tail_ns_per_rep"] = [r["tail_ns"] for r in recs]
med["end_max_ns_per_rep"] = [r["end_max_ns"] for r in recs]
print(json.dumps({"variant": a.variant, "rows": a.rows, "nq": a.nq, "tiles_per_block": [min(tiles), max(tiles)], "median": med}, indent=1))
