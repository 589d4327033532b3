"""Dev check: the IVF centroid factor 1/sqrt(n2) on the GPU equals numpy float32 for every
n2 in [1, 2^24) reachable from int8 codes (via rfx_ivf_set_centroids on synthetic tables)."""
import sys
import numpy as np
import torch
sys.path[:0] = ["/root/repo", "/root/repo/rag-foundation_amd"]
import rfx.ivf as rivf

rng = np.random.default_rng(0)
bad = 0
for trial in range(8):
    qc = rng.integers(-127, 128, size=(16384, 256)).astype(np.int8)
    qc[:, rng.integers(0, 256, size=16384)] = 0
    scale = rng.integers(1, 128, size=(16384, 1))
    qc = np.clip((qc.astype(int) * scale) // 127, -127, 127).astype(np.int8)
    ix = rivf.IvfIndex(256, 16384)
    ix.set_centroids(torch.from_numpy(qc).cuda())
    _, fc = ix.centroids()
    n2 = (qc.astype(np.int64) ** 2).sum(1).astype(np.float32)
    ref = np.where(n2 > 0, np.float32(1) / np.sqrt(np.maximum(n2, 1)), 0).astype(np.float32)
    bad += int((fc.cpu().numpy().view(np.uint32) != ref.view(np.uint32)).sum())
print("mismatches:", bad)
