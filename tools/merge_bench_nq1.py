"""Dev tool: merge-kernel latency for ONE query (config-2 shape: 391 lists x 16 sorted
candidates) — all-empty floor, dense, and 90 % pruned."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import topk_merge  # noqa: E402

nl, kl, k = 391, 16, 10
rng = np.random.default_rng(0)
s = -np.sort(-rng.standard_normal((1, nl, kl)).astype(np.float32), axis=2).reshape(1, -1)
r = rng.integers(0, 100_000, size=(1, nl * kl)).astype(np.int32)
empty_s, empty_r = np.full_like(s, -np.inf), np.full_like(r, 0x7fffffff)
pr_s, pr_r = s.copy(), r.copy()
kth = -np.sort(-s, axis=1)[:, 10 * k][:, None]
pr_r[s < kth] = 0x7fffffff
pr_s[s < kth] = -np.inf
for name, (a, b) in {"empty": (empty_s, empty_r), "dense": (s, r), "pruned": (pr_s, pr_r)}.items():
    a, b = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    for _ in range(5):
        topk_merge(a, b, k, list_len=kl)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        topk_merge(a, b, k, list_len=kl)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us per merge (incl. launch)", flush=True)
