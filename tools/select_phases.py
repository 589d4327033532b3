"""Dev tool (debug library): where the two-pass scan's select kernel (k_screen.hip
screen_select_kernel) spends its time.  Runs the search (query quantiser, kernel 10, select, gated
fallback) on a synthetic bf16 corpus, then reads the select's per-block phase clocks of the last
launch (100-MHz wall clock, rfx_dbg_select_times) and prints, over the 256 blocks, the block start
skew and the median / max duration of each phase:
  1 candidates loaded + compacted, 2 a_k, 3 drops + survivors, 4 exact re-score, 5 rank (thread 0),
  6 the answer written."""
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
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
f = _lib.lib.rfx_dbg_select_times
f.argtypes = [ctypes.c_void_p]
f.restype = ctypes.c_int
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
ix.enable_screen(1)
q = synth_rows(1, 0, a.nq, 768, "bf16")
ws = torch.empty(ix.workspace_bytes(a.nq, a.k), dtype=torch.uint8, device="cuda")
out = []
for rep in range(a.reps):
    ix.search(q, a.k, workspace=ws)
    torch.cuda.synchronize()
    t = np.zeros((256, 8), dtype=np.uint64)
    _lib.check(f(t.ctypes.data))
    t = t[:min(a.nq, 256)].astype(np.int64)[:, [0, 1, 2, 3, 4, 6, 5]] * 10  # ns, chronological
    d = np.diff(t[:, :7], axis=1)
    out.append({"skew_ns": int(t[:, 0].max() - t[:, 0].min()), "span_ns": int(t[:, 6].max() - t[:, 0].min()),
                "block_ns_med": int(np.median(t[:, 6] - t[:, 0])), "block_ns_max": int((t[:, 6] - t[:, 0]).max()),
                "phase_ns_med": [int(x) for x in np.median(d, axis=0)],
                "phase_ns_max": [int(x) for x in d.max(axis=0)]})
diag, fb = ix.screen_diag(a.nq, a.k, ws)
best = sorted(out[a.reps // 2:], key=lambda o: o["span_ns"])[len(out[a.reps // 2:]) // 2]
print(json.dumps({"rows": a.rows, "nq": a.nq, "kept_mean": float(diag[:, 0].mean()),
                  "survivors_mean": float(diag[:, 1].mean()), "fallback": fb, "median_rep": best,
                  "phases": ["load+compact", "a_k", "drops+survivors", "re-score", "rank", "write"]}, indent=1))
