"""CPU: the IVF-Flat int8 restatement (oracle/ivf.py) — quantisation invariants, exhaustive-probe
search equals a brute-force scan of the same int8 scores, k-means determinism, and recall on a
clustered corpus.  (No reference counterpart exists: SURVEY §8 config 5 is an extension; the GPU
is held bit-exactly to this oracle in tests/test_gpu_ivf.py.)"""
import numpy as np

from oracle import ivf, search as osearch, synth


def test_quantize_invariants():
    x = synth.synth_rows(3, 0, 50, 256).astype(np.float32)
    x[7] = 0.0
    q, inv = ivf.quantize(x)
    assert q.dtype == np.int8 and (np.abs(q.astype(int)) <= 127).all()
    amax_pos = np.abs(x).argmax(axis=1)
    for i in range(50):
        if i == 7:
            assert inv[i] == 0 and not q[i].any()
        else:
            assert abs(int(q[i, amax_pos[i]])) == 127
            assert np.allclose(q[i] * inv[i], x[i], atol=inv[i] * 0.5 + 1e-9)


def test_clustered_rows_normalised_and_clustered():
    x = ivf.clustered_rows(100, 8, 1, 0, 400, 256).astype(np.float64)
    assert np.allclose((x * x).sum(1), 1.0, atol=1e-6)
    s = x @ x.T
    raw = ivf.clustered_raw(100, 8, 1, 0, 400, 256)
    assert raw.shape == (400, 256)
    # rows of the same centre are much closer than rows of different centres
    bn = synth.splitmix64_int(1)
    lab = ((synth.splitmix64(np.uint64(bn) + np.uint64(ivf.L_KEY) + np.arange(400, dtype=np.uint64))
            >> np.uint64(32)) % np.uint64(8)).astype(int)
    same = s[lab[:, None] == lab[None, :]].mean()
    diff = s[lab[:, None] != lab[None, :]].mean()
    assert same > 0.4 and abs(diff) < 0.1


def _small_index(n=3000, d=256, nlist=16, seed=5):
    rows = ivf.clustered_rows(7, 32, seed, 0, n, d)
    codes, inv = ivf.quantize(rows)
    qc, fc = ivf.train(codes[:: max(1, n // 1024)], nlist, iters=4)
    labels = ivf.assign(codes, qc, fc)
    return rows, codes, inv, qc, fc, labels


def test_exhaustive_probe_equals_bruteforce_on_codes():
    rows, codes, inv, qc, fc, labels = _small_index()
    qrows = ivf.clustered_rows(7, 32, 99, 0, 20, rows.shape[1])
    qq, qinv = ivf.quantize(qrows)
    s, r = ivf.search(qq, qinv, codes, inv, labels, qc, fc, nprobe=qc.shape[0], k=10)
    d = ivf.int_dot(qq, codes).astype(np.float32) * (inv[None, :] * qinv[:, None]).astype(np.float32)
    for i in range(20):
        o = np.lexsort((np.arange(len(inv)), -d[i]))[:10]
        assert np.array_equal(r[i], o) and np.array_equal(s[i], d[i, o])


def test_train_deterministic_and_lists_sorted():
    a = _small_index()
    b = _small_index()
    assert np.array_equal(a[3], b[3]) and np.array_equal(a[5], b[5])
    order, off = ivf.build_lists(a[5], 16)
    assert off[-1] == len(order) and (np.diff(off) >= 0).all()
    for l in range(16):
        seg = order[off[l]:off[l + 1]]
        assert (a[5][seg] == l).all() and (np.diff(seg) > 0).all()


def test_recall_on_clustered_corpus():
    rows, codes, inv, qc, fc, labels = _small_index(n=4000, nlist=32)
    qrows = ivf.clustered_rows(7, 32, 123, 0, 30, rows.shape[1])
    qq, qinv = ivf.quantize(qrows)
    _, r = ivf.search(qq, qinv, codes, inv, labels, qc, fc, nprobe=4, k=10)
    _, truth = osearch.topk(qrows.astype(np.float64), rows.astype(np.float64), 10)
    recall = np.mean([len(set(r[i]) & set(truth[i])) / 10 for i in range(30)])
    assert recall > 0.8, recall
