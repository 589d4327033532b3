"""Dev tool: time the top-k merge kernel on synthetic sorted candidate lists (nq 256, 512 lists of
KL per query, like the config-3 scan output) for list_len hints 1 and KL."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import topk_merge  # noqa: E402

nq, nl, kl, k = 256, 512, 10, 10
rng = np.random.default_rng(0)
s = -np.sort(-rng.standard_normal((nq, nl, kl)).astype(np.float32), axis=2).reshape(nq, -1)
r = rng.integers(0, 10_000_000, size=(nq, nl * kl)).astype(np.int32)
cs, cr = torch.from_numpy(s).cuda(), torch.from_numpy(r).cuda()
for ll in (1, kl, 1, kl):
    for _ in range(3):
        topk_merge(cs, cr, k, list_len=ll)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        topk_merge(cs, cr, k, list_len=ll)
    e1.record()
    torch.cuda.synchronize()
    print(f"list_len={ll}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per merge", flush=True)
