"""Diagnostic: final per-list pruning bounds of k_scan_mfma5.h (MODE 8192) against each query's true
10th-best score; any bound above it would prune a true top-10 row.  Dev tool, not product."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import synth as osynth  # noqa: E402
from rfx import _lib  # noqa: E402
from rfx.index import DeviceIndex, synth_rows  # noqa: E402

f = _lib.lib.rfx_dbg_scan_variant
f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
D, NQ, K = 768, 256, 10
st = _lib.stream_ptr()
rows = 100_003
ix = DeviceIndex(D, "bf16", 0)
ix.add_synthetic(7, rows)
x = torch.from_numpy(osynth.to_f64(osynth.synth_rows(7, 0, rows, D, "bf16"), "bf16")).cuda()
for qs in (9, 10):
    q = synth_rows(qs, 0, NQ, D, "bf16")
    qf = torch.from_numpy(osynth.to_f64(osynth.synth_rows(qs, 0, NQ, D, "bf16"), "bf16")).cuda()
    S = qf @ x.T
    top = torch.topk(S, 12, dim=1)
    ref = top.values[:, K - 1]
    _, ncand = ix.plan(NQ, K)
    ws = torch.zeros(ix.workspace_bytes(NQ, K), dtype=torch.uint8, device="cuda")
    cs = torch.full((NQ, ncand), -np.inf, dtype=torch.float32, device="cuda")
    cr = torch.full((NQ, ncand), -1, dtype=torch.int32, device="cuda")
    _lib.check(f(ix.handle, _lib.ptr(q), NQ, K, 1000 + 8192, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
    torch.cuda.synchronize()
    nl = 512
    thr = cs.flatten()[: NQ * nl].view(NQ, nl).double()
    fromtau = cr.flatten()[: NQ * nl].view(NQ, nl)
    bad = thr > ref[:, None] + 1e-6
    print(f"qseed={qs}: lane bounds above the true 10th best: {int(bad.sum())} (queries {int(bad.any(1).sum())})")
    for qi in torch.nonzero(bad.any(1)).flatten()[:4].tolist():
        li = torch.nonzero(bad[qi]).flatten()[:4].tolist()
        print(f"  q{qi}: ref10 {float(ref[qi]):.6f} top12 {[round(v, 6) for v in top.values[qi].tolist()]}")
        print(f"    lists {li} bounds {[round(float(thr[qi, l]), 6) for l in li]} from_tau {[int(fromtau[qi, l]) for l in li]}")
    tw = 16
    nq_pad = 256
    tau_off = (nq_pad * D * 2 + 255) // 256 * 256
    tab = ws[tau_off: tau_off + nq_pad * tw * 4].view(torch.int32).view(nq_pad, tw).cpu().numpy().view(np.uint32)
    o = tab[:, :10]
    fl = np.where(o & 0x80000000, o & 0x7fffffff, ~o & 0xffffffff).astype(np.uint32).view(np.float32)
    for qi in torch.nonzero(bad.any(1)).flatten()[:4].tolist():
        print(f"    q{qi} table slots {np.round(fl[qi].astype(np.float64), 6).tolist()}")
