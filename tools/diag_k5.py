"""Diagnostic: miss statistics of k_scan_mfma5.h variants over several seeds/sizes (bf16, d 768,
nq 256, k 10) against the oracle.  Dev tool, not product."""
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
modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "1000,20,1512,3048,5096").split(",")]
st = _lib.stream_ptr()
tot = {m: 0 for m in modes}
for rows in (60_000, 100_003):
    ix = DeviceIndex(D, "bf16", 0)
    ix.add_synthetic(7, rows)
    x = torch.from_numpy(osynth.to_f64(osynth.synth_rows(7, 0, rows, D, "bf16"), "bf16")).cuda()
    for qs in (8, 9, 10, 11):
        q = synth_rows(qs, 0, NQ, D, "bf16")
        qf = torch.from_numpy(osynth.to_f64(osynth.synth_rows(qs, 0, NQ, D, "bf16"), "bf16")).cuda()
        S = qf @ x.T
        ref = torch.topk(S, K, dim=1).values[:, K - 1]  # 10th best score (f64)
        _, ncand = ix.plan(NQ, K)
        ws = torch.zeros(ix.workspace_bytes(NQ, K), dtype=torch.uint8, device="cuda")
        for m in modes:
            cs = torch.full((NQ, ncand), -np.inf, dtype=torch.float32, device="cuda")
            cr = torch.full((NQ, ncand), 0x7fffffff, dtype=torch.int32, device="cuda")
            _lib.check(f(ix.handle, _lib.ptr(q), NQ, K, m, _lib.ptr(cs), _lib.ptr(cr), _lib.ptr(ws), ws.numel(), st))
            torch.cuda.synchronize()
            if m == 20:  # v4's own list layout
                nt = (rows + 31) // 32
                tpb = (nt + min(256, nt) - 1) // min(256, nt)
                w4 = ((nt + tpb - 1) // tpb) * 2 * 10
                cs = cs.flatten()[: NQ * w4].view(NQ, w4)
                cr = cr.flatten()[: NQ * w4].view(NQ, w4)
            # every row whose oracle score reaches the 10th best must be among the candidates
            need = S >= (ref[:, None] - 1e-9)
            ok = (cr >= 0) & (cr < rows) & torch.isfinite(cs)
            have = torch.zeros_like(need)
            have.scatter_(1, cr.long().clamp(0, rows - 1), ok)
            miss = int((need & ~have).sum())
            if miss and m == 1000:
                for qi, ri in torch.nonzero(need & ~have).tolist()[:6]:
                    t = ri // 32
                    print(f"    q{qi} row {ri}: tile {t} it {t // 256} block {t % 256} in-tile {ri % 32} "
                          f"score {float(S[qi, ri]):.6f} ref10 {float(ref[qi]):.6f}")
            # candidate scores against the oracle score of the same row
            sc = S.gather(1, cr.long().clamp(0, rows - 1)).float()
            err = (cs - sc).abs().masked_fill(~ok, 0)
            nbad = int((err > 1e-5).sum())
            if nbad:
                qi, ci = torch.nonzero(err > 1e-5)[0].tolist()
                ri = int(cr[qi, ci])
                print(f"    mode={m}: {nbad} candidate scores off by > 1e-5, e.g. q{qi} row {ri} (tile {ri // 32} "
                      f"in-tile {ri % 32}) got {float(cs[qi, ci]):.6f} want {float(sc[qi, ci]):.6f}")
            tot[m] += miss
            print(f"rows={rows} qseed={qs} mode={m}: missing top-10 rows {miss}", flush=True)
print("TOTAL", tot)
