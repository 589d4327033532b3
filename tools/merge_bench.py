"""Dev tool: time the top-k merge kernel on synthetic sorted candidate lists (nq 256, 512 lists of
KL per query, like the config-3 scan output) for list_len hints 1 and KL, dense lists and the
sparse lists the v5 scan writes (entries below the final bound dropped)."""
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
sp_s, sp_r = s.copy(), r.copy()
kth = -np.sort(-s, axis=1)[:, 2 * k][:, None]
sp_r[s < kth] = 0x7fffffff
sp_s[s < kth] = -np.inf
cases = {"dense": (torch.from_numpy(s).cuda(), torch.from_numpy(r).cuda()),
         "sparse": (torch.from_numpy(sp_s).cuda(), torch.from_numpy(sp_r).cuda())}
for name, (a, b) in cases.items():
    for ll in (1, kl):
        for _ in range(3):
            topk_merge(a, b, k, list_len=ll)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            topk_merge(a, b, k, list_len=ll)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name} list_len={ll}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per merge", flush=True)
