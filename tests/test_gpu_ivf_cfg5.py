"""GPU parity of the IVF-Flat int8 path at config 5's real shape (BASELINE.json configs[4]:
nlist 4096, nprobe 32, batches of 256 queries, top-10, d 768) on a clustered 1M-row corpus — the
per-GPU list geometry of the 8-GPU config (12.5M rows / 4096 lists) at 1/12 of the rows, so the
CPU oracle (oracle/ivf.py, f64-BLAS integer dots) finishes in tens of seconds.

Every stage is held BIT-EXACT to the oracle, as in tests/test_gpu_ivf.py: int8 codes and scales of
all rows, the k-means centroids (65,536-row sample, 16 per list), the list of every row, the
posting lists, and the scores and rows of all 256 queries.  Then the quality metric of config 5:
recall@10 against the exact brute-force top-10 of the oracle (oracle.search.topk_blocks, f64
rescoring) for every 4th query, with and without the exact re-rank (measured 0.8625 / 0.8719 at
this 4-iteration, 16-rows-per-list training; tools/bench_ivf.py's 262k-row, 10-iteration training
of the full shard is the serving configuration).  Reference seam:
gemini_rag.py:463-469 (the file-search tool the index answers)."""
import numpy as np
import pytest
import torch

from oracle import ivf as oivf
from oracle import search as osearch
from oracle import synth as osynth

pytestmark = pytest.mark.gpu

N, DIM, NLIST, NPROBE, NQ, K = 1 << 20, 768, 4096, 32, 256, 10
CSEED, CENTRES, SEED, QSEED = 1234, 16384, 1, 2  # tools/bench_ivf.py's corpus
TRAIN_STEP, ITERS = 16, 4
BLK = 1 << 16


def to_np(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


@pytest.fixture(scope="module")
def cfg5():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    from rfx.ivf import IvfIndex, synth_clustered
    rows = synth_clustered(CSEED, CENTRES, SEED, 0, N, DIM, "bf16")
    ix = IvfIndex(DIM, NLIST)
    ix.train(rows[::TRAIN_STEP].contiguous(), iters=ITERS)
    ix.add(rows)
    ix.build()
    q = synth_clustered(CSEED, CENTRES, QSEED, 0, NQ, DIM, "bf16")
    torch.cuda.synchronize()
    rows_np = to_np(rows)
    # oracle quantiser, block by block (1M x 768 f32 at once would be 3 GB per temporary)
    codes = np.empty((N, DIM), dtype=np.int8)
    inv = np.empty(N, dtype=np.float32)
    for b in range(0, N, BLK):
        codes[b:b + BLK], inv[b:b + BLK] = oivf.quantize(oivf.stored_to_f32(rows_np[b:b + BLK], "bf16"))
    sq, _ = oivf.quantize(oivf.stored_to_f32(rows_np[::TRAIN_STEP], "bf16"))
    qc, fc = oivf.train(sq, NLIST, ITERS)
    return {"ix": ix, "rows": rows, "rows_np": rows_np, "q": q, "codes": codes, "inv": inv, "qc": qc, "fc": fc}


@pytest.mark.timeout(600)
def test_cfg5_codes_centroids_lists_bit_exact(cfg5):
    ix = cfg5["ix"]
    gc, ginv, glab = ix.codes()
    assert np.array_equal(gc.cpu().numpy(), cfg5["codes"]), "int8 codes differ"
    assert np.array_equal(ginv.cpu().numpy().view(np.uint32), cfg5["inv"].view(np.uint32)), "row scales differ"
    gqc, gfc = ix.centroids()
    assert np.array_equal(gqc.cpu().numpy(), cfg5["qc"]), "k-means centroids differ"
    assert np.array_equal(gfc.cpu().numpy().view(np.uint32), cfg5["fc"].view(np.uint32))
    lab = oivf.assign(cfg5["codes"], cfg5["qc"], cfg5["fc"])
    assert np.array_equal(glab.cpu().numpy(), lab), "list assignment differs"
    cfg5["labels"] = lab
    off, ids = ix.lists()
    order, ref_off = oivf.build_lists(lab, NLIST)
    assert np.array_equal(off.cpu().numpy(), ref_off) and np.array_equal(ids.cpu().numpy(), order)
    sizes = np.diff(ref_off)
    assert (sizes > 0).sum() > NLIST // 2, "degenerate clustering: most lists empty"


@pytest.mark.timeout(600)
def test_cfg5_search_bit_exact(cfg5):
    lab = cfg5.get("labels")
    if lab is None:
        lab = oivf.assign(cfg5["codes"], cfg5["qc"], cfg5["fc"])
    ix, q = cfg5["ix"], cfg5["q"]
    s, r = ix.search(q, K, NPROBE)
    qq, qinv = oivf.quantize(oivf.stored_to_f32(to_np(q), "bf16"))
    ref_s, ref_r = oivf.search(qq, qinv, cfg5["codes"], cfg5["inv"], lab, cfg5["qc"], cfg5["fc"], NPROBE, K)
    assert np.array_equal(r.cpu().numpy(), ref_r), "IVF rows differ from the oracle"
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32)), "IVF scores differ"
    assert (ref_r >= 0).all()


@pytest.mark.timeout(600)
def test_cfg5_recall_vs_oracle_bruteforce(cfg5):
    ix, q, rows_np = cfg5["ix"], cfg5["q"], cfg5["rows_np"]
    sel = np.arange(0, NQ, 4)
    q64 = osynth.to_f64(to_np(q)[sel], "bf16")

    def blocks():
        for b in range(0, N, BLK):
            yield b, oivf.stored_to_f32(rows_np[b:b + BLK], "bf16")

    _, exact = osearch.topk_blocks(q64, blocks(), K)
    _, r_ivf = ix.search(q, K, NPROBE)
    _, r_rr = ix.search_rerank(q, K, NPROBE, cfg5["rows"])
    rec = lambda rr: float(np.mean([len(set(rr[i].tolist()) & set(exact[j].tolist())) / K for j, i in enumerate(sel)]))
    r_ivf, r_rr = r_ivf.cpu().numpy(), r_rr.cpu().numpy()
    print(f"cfg5 recall@{K}: ivf {rec(r_ivf):.4f}  rerank {rec(r_rr):.4f}")
    # measured (round 3, this corpus and training): ivf 0.8625, rerank 0.8719 — the misses are rows
    # in lists outside the 32 probed (a quality property of IVF, not a parity one); the floor below
    # catches a broken probe / list build, which drops recall far lower
    assert rec(r_ivf) >= 0.8 and rec(r_rr) >= rec(r_ivf), (rec(r_ivf), rec(r_rr))
