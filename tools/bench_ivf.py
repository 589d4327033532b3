"""IVF-Flat int8 benchmark (BASELINE.json configs[4], per-GPU shard): 100M × 768 over 8 GPUs =
12.5M rows per GPU, nlist 4096, nprobe 32, batches of 256 queries, top-10.  Clustered synthetic
corpus (oracle/ivf.py clustered_rows: 16384 centres + equal-energy noise), rows generated in
chunks on the device, k-means on the first 262,144 rows (64 per list), then quantise + assign all
rows and build the posting lists.  Reports build times, search QPS, the probed-list bytes per
batch against HBM peak, and recall@10 against the exact bf16 brute-force search of the same rows.

Usage: python tools/bench_ivf.py [--rows R] [--nlist L] [--nprobe P] [--nq Q] [--k K] [--steps S]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import DeviceIndex  # noqa: E402
from rfx.ivf import IvfIndex, synth_clustered  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=12_500_000)
ap.add_argument("--dim", type=int, default=768)
ap.add_argument("--nlist", type=int, default=4096)
ap.add_argument("--nprobe", type=int, default=32)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--centres", type=int, default=16384)
ap.add_argument("--train-rows", type=int, default=262_144)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--no-recall", action="store_true")
ap.add_argument("--rerank-k", type=int, default=16)
a = ap.parse_args()

torch.cuda.set_device(0)
CSEED, SEED, QSEED, CHUNK = 1234, 1, 2, 1 << 20


def t():
    torch.cuda.synchronize()
    return time.perf_counter()


ix = IvfIndex(a.dim, a.nlist)
t0 = t()
ix.train(synth_clustered(CSEED, a.centres, SEED, 0, a.train_rows, a.dim, "bf16"), iters=a.iters)
t1 = t()
for r0 in range(0, a.rows, CHUNK):
    ix.add(synth_clustered(CSEED, a.centres, SEED, r0, min(CHUNK, a.rows - r0), a.dim, "bf16"))
t2 = t()
ix.build()
t3 = t()
print(f"train {t1 - t0:.2f}s  add {t2 - t1:.2f}s  build {t3 - t2:.2f}s", flush=True)

q = synth_clustered(CSEED, a.centres, QSEED, 0, a.nq, a.dim, "bf16")
ws = torch.empty(ix.workspace_bytes(a.nq, a.k, a.nprobe), dtype=torch.uint8, device="cuda")
for _ in range(3):
    s, r = ix.search(q, a.k, a.nprobe, workspace=ws)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(a.steps):
    s, r = ix.search(q, a.k, a.nprobe, workspace=ws)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.steps

# bytes the posting-list scan must read per batch: every probed list once (codes + scale + id)
off, _ = ix.lists()
sizes = (off[1:] - off[:-1]).cpu()
# the batch's probed lists, recomputed outside the timed region (int8 dots are exact in f32)
qc, fc = ix.centroids()
from rfx.ivf import quantize  # noqa: E402
qq, _ = quantize(q)
scores = (qq.float() @ qc.float().T) * fc[None, :]
probes = torch.topk(scores, a.nprobe, dim=1).indices.unique().cpu()
list_bytes = int(sizes[probes].sum()) * (a.dim + 8)
gbps = list_bytes / (ms * 1e-3) / 1e9
out = {"metric": "IVF-Flat int8 top-k QPS (config 5 per-GPU shard)", "value": round(a.nq / (ms * 1e-3), 1),
       "unit": "queries/s", "ms_per_batch": round(ms, 4), "rows": a.rows, "dim": a.dim, "nlist": a.nlist,
       "nprobe": a.nprobe, "nq": a.nq, "k": a.k, "probed_lists": int(len(probes)),
       "probed_list_bytes": list_bytes, "achieved_list_GBps": round(gbps, 1),
       "build_s": {"train": round(t1 - t0, 2), "add": round(t2 - t1, 2), "lists": round(t3 - t2, 2)}}

if not a.no_recall:
    # the original rows, once, for the exact brute-force reference and the re-rank variant
    full = torch.empty((a.rows, a.dim), dtype=torch.bfloat16, device="cuda")
    for r0 in range(0, a.rows, CHUNK):
        full[r0:r0 + CHUNK] = synth_clustered(CSEED, a.centres, SEED, r0, min(CHUNK, a.rows - r0), a.dim, "bf16")
    bf = DeviceIndex(a.dim, "bf16", capacity=a.rows)
    bf.add(full)
    _, rb = bf.search(q, a.k)
    rb = rb.cpu().tolist()
    rec = lambda rr: round(sum(len(set(x) & set(y)) for x, y in zip(rr.cpu().tolist(), rb)) / (a.k * a.nq), 4)
    out["recall_at_k"] = rec(r)
    bf.close()
    rk = a.rerank_k
    for _ in range(3):
        _, r2 = ix.search_rerank(q, a.k, a.nprobe, full, rerank_k=rk)
    e0.record()
    for _ in range(a.steps):
        _, r2 = ix.search_rerank(q, a.k, a.nprobe, full, rerank_k=rk)
    e1.record()
    torch.cuda.synchronize()
    ms2 = e0.elapsed_time(e1) / a.steps
    out["rerank"] = {"rerank_k": rk, "recall_at_k": rec(r2), "ms_per_batch": round(ms2, 4),
                     "value": round(a.nq / (ms2 * 1e-3), 1)}
print(json.dumps(out), flush=True)
