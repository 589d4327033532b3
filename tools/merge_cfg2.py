"""Dev tool: merge-kernel cost on the REAL config-2 scan output (100k x 768 f32, nq 1, k 10):
list_len 1 vs the scan's list length, and the live-candidate count after the scan's pruning."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import DeviceIndex, synth_rows, topk_merge  # noqa: E402

ix = DeviceIndex(768, "f32", 0, capacity=100_000)
ix.add_synthetic(0, 100_000)
q = synth_rows(1, 0, 1, 768, "f32")
cs, cr = ix.scan(q, 10)
torch.cuda.synchronize()
live = int(((cr != 0x7fffffff) & torch.isfinite(cs)).sum())
print(f"candidates {cs.shape[1]}, live after scan pruning {live}, list_len {ix.list_len(1, 10)}", flush=True)
for ll in (1, ix.list_len(1, 10)):
    for _ in range(5):
        topk_merge(cs, cr, 10, list_len=ll)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(100):
        topk_merge(cs, cr, 10, list_len=ll)
    e1.record()
    torch.cuda.synchronize()
    print(f"list_len {ll}: {e0.elapsed_time(e1) / 100 * 1e3:.1f} us per merge (incl. launch)", flush=True)

# host view of the admission bound the merge computes (tail / carried bound per list, max)
import numpy as np  # noqa: E402
s_np, r_np = cs.cpu().numpy()[0], cr.cpu().numpy()[0]
ll, k = ix.list_len(1, 10), 10
T = -np.inf
for j in range(len(s_np) // ll):
    ss, rr = s_np[j * ll: j * ll + k], r_np[j * ll: j * ll + k]
    live = rr != 0x7fffffff
    t = ss.min() if live.all() else (ss[~live & np.isfinite(ss)].max() if (~live & np.isfinite(ss)).any() else -np.inf)
    T = max(T, t)
adm = int(((r_np != 0x7fffffff) & (s_np >= T)).sum())
print(f"T = {T:.6f}; live candidates >= T: {adm}; true 10th best {np.sort(s_np[r_np != 0x7fffffff])[-10]:.6f}", flush=True)
