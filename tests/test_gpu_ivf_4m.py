"""GPU parity of the IVF-Flat int8 path at 4M rows: a third of config 5's per-GPU shard
(12.5M rows / 4096 lists; BASELINE.json configs[4]) held to the CPU oracle (oracle/ivf.py), with the oracle
running block by block so it fits the host in memory and time.

- int8 codes and row scales of ALL 4,194,304 rows bit-exact (oracle quantiser in 64k-row blocks);
- the k-means centroids bit-exact (65,536-row strided sample, 4 iterations);
- the list of every 8th row bit-exact (oracle assignment in blocks; 524,288 rows x 4096 lists);
- the posting lists are the stable sort of the device's labels (offsets and order), and the scores and rows
  of all 256 queries equal the oracle's IVF search over them (nprobe 32, top-10), bit for bit.

Reference seam: gemini_rag.py:463-469 (the file-search tool the index answers)."""
import numpy as np
import pytest
import torch

from oracle import ivf as oivf

pytestmark = pytest.mark.gpu

N, DIM, NLIST, NPROBE, NQ, K = 4 << 20, 768, 4096, 32, 256, 10
CSEED, CENTRES, SEED, QSEED = 1234, 16384, 1, 2  # tools/bench_ivf.py's corpus
TRAIN_STEP, ITERS = 64, 4
LAB_STEP = 8
BLK = 1 << 16


def to_np(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


@pytest.fixture(scope="module")
def ivf4m():
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
    del rows
    yield {"ix": ix, "rows_np": rows_np, "q": q}
    ix.close()


@pytest.mark.timeout(600)
def test_ivf4m_codes_and_centroids_bit_exact(ivf4m):
    ix, rows_np = ivf4m["ix"], ivf4m["rows_np"]
    gc, ginv, glab = ix.codes()
    gc, ginv = gc.cpu().numpy(), ginv.cpu().numpy()
    for b in range(0, N, BLK):  # the oracle quantiser block by block (4M x 768 f32 at once would be 12 GB)
        c, inv = oivf.quantize(oivf.stored_to_f32(rows_np[b:b + BLK], "bf16"))
        assert np.array_equal(gc[b:b + BLK], c), f"int8 codes differ in rows [{b}, {b + BLK})"
        assert np.array_equal(ginv[b:b + BLK].view(np.uint32), inv.view(np.uint32)), f"row scales differ at {b}"
    sq, _ = oivf.quantize(oivf.stored_to_f32(rows_np[::TRAIN_STEP], "bf16"))
    qc, fc = oivf.train(sq, NLIST, ITERS)
    gqc, gfc = ix.centroids()
    assert np.array_equal(gqc.cpu().numpy(), qc), "k-means centroids differ"
    assert np.array_equal(gfc.cpu().numpy().view(np.uint32), fc.view(np.uint32))
    ivf4m.update(codes=gc, inv=ginv, qc=qc, fc=fc, labels=glab.cpu().numpy())


@pytest.mark.timeout(600)
def test_ivf4m_lists_and_search_bit_exact(ivf4m):
    if "labels" not in ivf4m:
        pytest.skip("needs test_ivf4m_codes_and_centroids_bit_exact")
    ix, q = ivf4m["ix"], ivf4m["q"]
    codes, inv, qc, fc, lab = (ivf4m[x] for x in ("codes", "inv", "qc", "fc", "labels"))
    # the list of every 8th row against the oracle's assignment (blocks of 64k rows inside oivf.assign)
    sel = np.arange(0, N, LAB_STEP)
    assert np.array_equal(lab[sel], oivf.assign(codes[sel], qc, fc)), "list assignment differs"
    off, ids = ix.lists()
    order, ref_off = oivf.build_lists(lab, NLIST)
    assert np.array_equal(off.cpu().numpy(), ref_off) and np.array_equal(ids.cpu().numpy(), order)
    assert (np.diff(ref_off) > 0).sum() > NLIST // 2, "degenerate clustering: most lists empty"
    s, r = ix.search(q, K, NPROBE)
    qq, qinv = oivf.quantize(oivf.stored_to_f32(to_np(q), "bf16"))
    ref_s, ref_r = oivf.search(qq, qinv, codes, inv, lab, qc, fc, NPROBE, K)
    assert np.array_equal(r.cpu().numpy(), ref_r), "IVF rows differ from the oracle"
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32)), "IVF scores differ"
    assert (ref_r >= 0).all()
