"""Diagnostic: 256-query-stationary kernels (v4 = k_scan_mfma4.h, v5 = k_scan_mfma5.h) against the
oracle on one small configuration, plus a validity check of the v5 threshold table (every query's
min over its KL slots must be <= its true KL-th best score).  Dev tool, not product."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import search as osearch  # noqa: E402
from oracle import synth as osynth  # noqa: E402
from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=50_000)
ap.add_argument("--nq", type=int, default=200)
ap.add_argument("--dtype", default="f16")
ap.add_argument("--ks", default="1,2,3,4,5,10")
a = ap.parse_args()
f = _lib.lib.rfx_dbg_scan_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
D = 768
ix = DeviceIndex(D, a.dtype, 0)
ix.add_synthetic(7, a.rows)
q = synth_rows(8, 0, a.nq, D, a.dtype)
x64 = osynth.to_f64(osynth.synth_rows(7, 0, a.rows, D, a.dtype), a.dtype)
q64 = osynth.to_f64(osynth.synth_rows(8, 0, a.nq, D, a.dtype), a.dtype)
S = q64 @ x64.T
st = _lib.stream_ptr()
nq_pad = (a.nq + 255) // 256 * 256
tau_off = (nq_pad * D * 2 + 255) // 256 * 256
for k in [int(v) for v in a.ks.split(",")]:
    kl = 4 if k <= 4 else 10
    ref_s, ref_r = osearch.topk(q64, x64, k)
    _, ncand = ix.plan(a.nq, k)
    ws = torch.zeros(ix.workspace_bytes(a.nq, k), dtype=torch.uint8, device="cuda")
    runs = [("v4", 20), ("v5", 1000)]
    if kl == 10:
        runs += [("v5-notau", 1512), ("v5-noprune", 2024)]
    for name, mode in runs:
        cs = torch.full((a.nq, ncand), -np.inf, dtype=torch.float32, device="cuda")
        cr = torch.full((a.nq, ncand), 0x7fffffff, dtype=torch.int32, device="cuda")
        _lib.check(f(ix.handle, _lib.ptr(q), a.nq, k, mode, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
        torch.cuda.synchronize()
        s_np, r_np = cs.cpu().numpy(), cr.cpu().numpy().astype(np.int64)
        if name == "v4":  # v4's own list count (its plan: contiguous ranges of ceil(ntiles / 256) tiles)
            nt = (a.rows + 31) // 32
            tpb = (nt + min(256, nt) - 1) // min(256, nt)
            w4 = ((nt + tpb - 1) // tpb) * 2 * kl
            s_np = s_np.reshape(-1)[: a.nq * w4].reshape(a.nq, w4)
            r_np = r_np.reshape(-1)[: a.nq * w4].reshape(a.nq, w4)
        bad = 0
        for i in range(a.nq):
            order = np.lexsort((r_np[i], -s_np[i].astype(np.float64)))[:k]
            got = r_np[i][order]
            if not np.array_equal(got, ref_r[i]):
                bad += 1
                miss = sorted(set(ref_r[i].tolist()) - set(got.tolist()))
                print(f"  {name} k={k} q{i} missing rows {miss} tiles {[m // 32 for m in miss]}")
                if bad <= 1:
                    print(f"  {name} k={k} q{i}: got {got.tolist()} want {ref_r[i].tolist()} "
                          f"got_s {S[i, np.clip(got, 0, a.rows - 1)].round(5).tolist()} want_s {ref_s[i].round(5).tolist()}")
        msg = f"{name} k={k} kl={kl}: {bad}/{a.nq} queries differ"
        if name.startswith("v5"):
            tw = 16
            tab = ws[tau_off: tau_off + nq_pad * tw * 4].view(torch.int32).view(nq_pad, tw).cpu().numpy().view(np.uint32)
            o = tab[: a.nq, :kl].min(axis=1)
            # unord
            f32 = np.where(o & 0x80000000, o & 0x7fffffff, ~o & 0xffffffff).astype(np.uint32).view(np.float32)
            f32 = np.where(o == 0, -np.inf, f32)
            kth = np.sort(S, axis=1)[:, ::-1][:, kl - 1]
            viol = int((f32 > kth + 1e-6).sum())
            msg += f"; tau-table violations {viol}"
            if viol:
                i = int(np.nonzero(f32 > kth + 1e-6)[0][0])
                print("  q", i, "slots", tab[i, :kl].tolist(), "min", f32[i], "kth", kth[i],
                      "top", np.sort(S[i])[::-1][:kl].round(5).tolist())
        print(msg, flush=True)
