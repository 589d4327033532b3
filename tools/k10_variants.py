"""Dev tool (debug library): time kernel 10 (the two-pass scan's int8 screen) variants on the cfg3
corpus in bursts of back-to-back launches, variants interleaved over rounds (the chip's clock
settles per workload; cdna_hip_programming.md §5.4 rule 24).

variant = 10**8 * RING + MODE (k10_dbg.hip; round 5 first used 10**7 * RING + MODE, round 4 100000 * RING + MODE, round 3 1000 * RING + MODE): RING in {4, 6, 8, 10, 12}; MODE 1 = no top-k fold,
8 = no corpus stream after the prologue, 9 = both; 32 = count slow-path entries (reported, not
timed); 64 = the store-wide integer fast-path bound."""
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
ap.add_argument("--variants", default="1010485760,800000000,1010485761,1010486272")
ap.add_argument("--seconds", type=float, default=0.0, help="one variant back to back for this long (power sampling)")
ap.add_argument("--validate", action="store_true", help="each variant's two-pass answer must equal production's")
a = ap.parse_args()
f = _lib.lib.rfx_dbg_screen_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_size_t, ctypes.c_void_p]
f.restype = ctypes.c_int
ix = DeviceIndex(768, "bf16", 0, capacity=a.rows)
ix.add_synthetic(0, a.rows)
ix.enable_screen(1)
q = synth_rows(1, 0, a.nq, 768, "bf16")
ws = torch.empty(ix.workspace_bytes(a.nq, a.k), dtype=torch.uint8, device="cuda")
st = _lib.stream_ptr()
variants = [int(v) for v in a.variants.split(",")]


def launch(v):
    _lib.check(f(ix.handle, _lib.ptr(q), a.nq, a.k, v, _lib.ptr(ws), ws.numel(), st))


t_first = {}
for v in variants:  # warm + validate every variant launches (and time one cold launch: a bounded spin gone
    # wrong would show here as tens of ms before any burst)
    t0 = time.perf_counter()
    launch(v)
    torch.cuda.synchronize()
    t_first[v] = round((time.perf_counter() - t0) * 1e3, 3)
print(json.dumps({"first_launch_ms": t_first}), flush=True)
if a.validate:  # every variant's two-pass answer (no fallback) against the production search
    vs = _lib.lib.rfx_dbg_screen_search
    vs.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    vs.restype = ctypes.c_int
    ref_s, ref_r = ix.search(q, a.k)
    for v in variants:
        if (v % 10000000) & (1 | 8 | 512):  # timing-only variants (wrong results by design)
            continue
        s_ = torch.empty_like(ref_s)
        r_ = torch.empty_like(ref_r)
        fb = ctypes.c_uint32()
        _lib.check(vs(ix.handle, _lib.ptr(q), a.nq, a.k, v, _lib.ptr(s_), _lib.ptr(r_), _lib.ptr(ws), ws.numel(), st,
                      ctypes.byref(fb)))
        same = bool(torch.equal(r_, ref_r) and torch.equal(s_, ref_s))
        print(json.dumps({"variant": v, "equal_to_production": same, "fallback": bool(fb.value)}), flush=True)
        if not same:
            sys.exit(f"variant {v} differs from the production search")
if a.rounds == 0:
    sys.exit(0)
if a.seconds > 0:  # steady state of ONE variant (rocm-smi samples power / sclk meanwhile)
    v = variants[0]
    print(f"burst start {v}", file=sys.stderr, flush=True)  # (tools/r06/gpu_power.sh samples rocm-smi from here)
    n, t0 = 0, time.time()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    while time.time() - t0 < a.seconds:
        for _ in range(20):
            launch(v)
        n += 20
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"variant": v, "launches": n, "ms_per_launch": round(e0.elapsed_time(e1) / n, 4)}))
    sys.exit(0)
cnt = _lib.lib.rfx_dbg_screen_counts
cnt.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
cnt.restype = ctypes.c_int
for v in [v for v in variants if (v % 10000000) & 32]:  # slow-path entries of one launch (MODE 32 counter)
    launch(v)
    torch.cuda.synchronize()
    n = ctypes.c_uint64()
    _lib.check(cnt(ix.handle, a.nq, a.k, _lib.ptr(ws), ctypes.byref(n)))
    ntiles = -(-a.rows // 32)
    print(json.dumps({"variant": v, "slow_path_wave_entries": n.value, "wave_tiles": ntiles * 8,
                      "frac": round(n.value / (ntiles * 8), 5)}))
variants = [v for v in variants if not (v % 10000000) & 32]
res = {v: [] for v in variants}
for rnd in range(a.rounds):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        for _ in range(5):
            launch(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.burst):
            launch(v)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / a.burst)
out = {str(v): {"ms_per_launch_min": round(min(t), 4), "ms_per_launch_med": round(sorted(t)[len(t) // 2], 4)}
       for v, t in res.items()}
print(json.dumps({"rows": a.rows, "nq": a.nq, "burst": a.burst, "rounds": a.rounds, "variants": out}, indent=1))
