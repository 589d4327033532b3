"""Dev tool: how far below the true k-th best score a slot-table pruning bound sits.
10M Gaussian scores, 512 lists (kernel 10's (workgroup, half) lists of 32-row tiles), each list's
best published to slot list % S; bound = min over k slots (S = k, kernel 6) or the k-th largest of S
slots.  Prints the mean number of rows at or above the bound (k = 10 would be exact)."""
import numpy as np

rng = np.random.default_rng(1)
N, k = 10_000_000, 10
res = {}
for trial in range(5):
    s = rng.standard_normal(N).astype(np.float32)
    r = np.arange(N)
    lst = ((r // 32) % 256) * 2 + ((r % 32) >= 16)
    best = np.full(512, -np.inf, np.float32)
    np.maximum.at(best, lst, s)
    for S in (10, 16, 32, 64):
        sm = np.full(S, -np.inf, np.float32)
        np.maximum.at(sm, np.arange(512) % S, best)
        b = np.min(sm[:k]) if S == k else np.sort(sm)[-k]
        res.setdefault(S, []).append(int((s >= b).sum()))
print({S: float(np.mean(v)) for S, v in res.items()})
