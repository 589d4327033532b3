"""Dev tool: where the config-2 merge's time goes.  Times 200 back-to-back merges (HIP events) on
(a) the real config-2 scan output, (b) the same arrays with every candidate dead, (c) the first 112
candidates only, (d) the real output with list_len 1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import DeviceIndex, synth_rows, topk_merge  # noqa: E402


def t(cs, cr, ll, n=200):
    for _ in range(5):
        topk_merge(cs, cr, 10, list_len=ll)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        topk_merge(cs, cr, 10, list_len=ll)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


ix = DeviceIndex(768, "f32", 0, capacity=100_000)
ix.add_synthetic(0, 100_000)
q = synth_rows(1, 0, 1, 768, "f32")
cs, cr = ix.scan(q, 10)
torch.cuda.synchronize()
L = ix.list_len(1, 10)
live = int(((cr != 0x7fffffff) & torch.isfinite(cs)).sum())
print(f"n_cand {cs.shape[1]} live {live} list_len {L}", flush=True)
print(f"(a) real: {t(cs, cr, L):.1f} us", flush=True)
print(f"(d) real, list_len 1: {t(cs, cr, 1):.1f} us", flush=True)
dead_s, dead_r = torch.full_like(cs, float('-inf')), torch.full_like(cr, 0x7fffffff)
print(f"(b) all dead: {t(dead_s, dead_r, L):.1f} us", flush=True)
print(f"(c) 112 cands: {t(cs[:, :112].contiguous(), cr[:, :112].contiguous(), L):.1f} us", flush=True)
print(f"(e) 16 cands: {t(cs[:, :16].contiguous(), cr[:, :16].contiguous(), L):.1f} us", flush=True)
