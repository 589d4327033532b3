"""Dev tool (debug library): where kernel 11 (k_screen_valu.hip, the two-pass scan of a few questions;
config 2: 100k x 768 f32, nq 1, k 10) spends its time.  Runs lone-question searches on rotating corpus
copies, then reads the per-block phase clocks of the last launch (100-MHz wall clock,
rfx_dbg_k11_times) and prints medians over the repetitions:
  per block (median / max over blocks): quantiser, row stream, block merge + record + arrival;
  the last block: records loaded, bound + drop check, survivors, re-score + rank, end;
  span = last block's end - first block's start;
  survivors of query 0 and how many of them had no exact key from the blocks' early re-score (the
  last block re-scored those itself), median and the fraction of searches with any."""
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
ap.add_argument("--rows", type=int, default=100_000)
ap.add_argument("--dtype", default="f32")
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--copies", type=int, default=4)
ap.add_argument("--reps", type=int, default=40)
a = ap.parse_args()
f = _lib.lib.rfx_dbg_k11_times
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
f.restype = ctypes.c_int
ixs = []
for c in range(a.copies):
    ix = DeviceIndex(768, a.dtype, 0, capacity=a.rows)
    ix.add_synthetic(0, a.rows)
    ix.enable_screen(1)
    ixs.append(ix)
assert ixs[0].search_plan(1, a.k) == 11
q = synth_rows(1, 0, 1, 768, a.dtype)
ws = torch.empty(ixs[0].workspace_bytes(1, a.k), dtype=torch.uint8, device="cuda")
recs = []
for rep in range(a.reps):
    ixs[rep % a.copies].search(q, a.k, workspace=ws)
    torch.cuda.synchronize()
    bt = np.zeros((1024, 4), dtype=np.uint64)
    lt = np.zeros(8, dtype=np.uint64)
    _lib.check(f(bt.ctypes.data, lt.ctypes.data))
    nb = int((bt[:, 3] > 0).sum())
    b = bt[:nb].astype(np.int64) * 10
    l = lt.astype(np.int64) * 10
    t0 = b[:, 0].min()
    d = np.diff(b, axis=1)
    recs.append({"blocks": nb, "start_skew_ns": int(b[:, 0].max() - t0),
                 "quant_ns": [int(np.median(d[:, 0])), int(d[:, 0].max())],
                 "stream_ns": [int(np.median(d[:, 1])), int(d[:, 1].max())],
                 "merge_record_ns": [int(np.median(d[:, 2])), int(d[:, 2].max())],
                 "last_arrival_after_start_ns": int(b[:, 3].max() - t0),
                 "last_block_ns": [int(x) for x in np.diff(l[:6])],
                 "span_ns": int(l[5] - t0), "survivors": int(lt[6]), "missing_keys": int(lt[7])})
keys = ["start_skew_ns", "last_arrival_after_start_ns", "span_ns", "survivors", "missing_keys"]
med = {k: int(np.median([r[k] for r in recs[a.reps // 4:]])) for k in keys}
for k in ["quant_ns", "stream_ns", "merge_record_ns", "last_block_ns"]:
    arr = np.array([r[k] for r in recs[a.reps // 4:]])
    med[k] = [int(x) for x in np.median(arr, axis=0)]
med["searches_with_missing_keys"] = float(np.mean([r["missing_keys"] > 0 for r in recs[a.reps // 4:]]))
print(json.dumps({"rows": a.rows, "dtype": a.dtype, "blocks": recs[-1]["blocks"], "median": med,
                  "last_block_phases": ["records loaded", "bound+drop check", "survivors", "re-score+rank", "end"]},
                 indent=1))
