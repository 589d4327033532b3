"""IVF-Flat int8 (build plan item 8) — the SPECIFICATION of the path's
numerics, written as plain numpy from the formulas below (a standard IVF-Flat with symmetric
per-row int8 quantisation and spherical k-means), not from the kernels; the HIP implementation
(rag-foundation_amd/csrc/k_ivf.hip) is held to it.  TEST INFRASTRUCTURE ONLY (tests/, smoke(),
bench.py's cpu_baseline); never imported by the product path.

The reference has no IVF (its retrieval runs inside Gemini): SURVEY §8 marks config 5 an extension
with "no reference counterpart", so parity is UNPINNED against the reference by construction: this
file defines the numerics and the GPU path is held to it BIT-EXACTLY.  The names in parentheses
below say which kernel implements each step.  Every step is integer arithmetic or a single correctly rounded f32 operation
(IEEE in numpy and via the __f*_rn intrinsics on the GPU), so there is no tolerance anywhere:

  quantize (rows and queries; k_ivf.hip quantize_kernel)
    amax = max_d |x_d| (f32);  s = 127 / amax;  q_d = clamp(rint(x_d * s), -127, 127) (int8)
    inv = amax / 127   (amax == 0: q = 0, inv = 0)
  centroid factor (centroid_finalize_kernel)
    f_c = 1 / sqrt(f32(sum_d qc_d^2))                        (0 for an all-zero centroid)
  coarse score of int8 vector x against centroid c (exact int dot, < 2^24 so exact in f32)
    cs(x, c) = f32(dot_i32(x, qc_c)) * f_c
  assignment: argmax_c cs(row, c), ties -> lowest c
  k-means (train_kernels): init qc_j = quantized sample row j * (n_train // nlist);
    each iteration: assign every sample row; sum_c = sum of its rows' int8 codes (int32),
    amax_c = max_d |sum_c,d|; if count_c > 0 and amax_c > 0:
      qc_c,d = clamp(rint(f32(sum_c,d) * (127 / f32(amax_c))), -127, 127)  (else qc_c unchanged)
  posting lists: rows ordered by (list, row id)
  search (nprobe, k): probes = top-nprobe centroids by cs(query, c) (score desc, c asc);
    fine score of row r for query q = f32(dot_i32(q, r)) * (inv_r * inv_q)
    result = top-k over the probed lists' rows by (score desc, row asc), padded (-inf, -1).
"""
import numpy as np

from . import synth

_F = np.float32


def quantize(x: np.ndarray):
    """f32/f64-exact rows [n][d] (any float dtype holding f32 values) -> (int8 [n][d], inv f32 [n])."""
    x = np.asarray(x, dtype=np.float32)
    amax = np.abs(x).max(axis=1) if x.shape[1] else np.zeros(x.shape[0], np.float32)
    amax = amax.astype(np.float32)
    nz = amax > 0
    s = np.zeros_like(amax)
    s[nz] = _F(127) / amax[nz]
    q = np.rint(x * s[:, None]).clip(-127, 127).astype(np.int8)
    inv = (amax / _F(127)).astype(np.float32)
    return q, inv


def stored_to_f32(rows: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "bf16":
        return synth.bf16_bits_to_f32(rows)
    return np.asarray(rows).astype(np.float32)


def centroid_factor(qc: np.ndarray) -> np.ndarray:
    n2 = (qc.astype(np.int64) ** 2).sum(axis=1).astype(np.float32)
    f = np.zeros(qc.shape[0], dtype=np.float32)
    nz = n2 > 0
    f[nz] = _F(1) / np.sqrt(n2[nz])
    return f


def int_dot(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Exact int8 x int8 dot products [na][nb] (f64 BLAS: every partial sum < 2^53)."""
    return (a.astype(np.float64) @ b.astype(np.float64).T).astype(np.int64)


def coarse_scores(x: np.ndarray, qc: np.ndarray, fc: np.ndarray) -> np.ndarray:
    return int_dot(x, qc).astype(np.float32) * fc[None, :]


def assign(x: np.ndarray, qc: np.ndarray, fc: np.ndarray, block: int = 1 << 15) -> np.ndarray:
    out = np.empty(x.shape[0], dtype=np.int32)
    for b in range(0, x.shape[0], block):
        s = coarse_scores(x[b:b + block], qc, fc)
        out[b:b + block] = np.argmax(s, axis=1)  # first maximum = lowest centroid id
    return out


def train(xq: np.ndarray, nlist: int, iters: int):
    """k-means on quantized sample rows xq (int8 [n][d]) -> (qc int8 [nlist][d], fc f32 [nlist])."""
    n = xq.shape[0]
    if n < nlist:
        raise ValueError("need at least nlist training rows")
    step = n // nlist
    qc = xq[np.arange(nlist) * step].copy()
    for _ in range(iters):
        fc = centroid_factor(qc)
        lab = assign(xq, qc, fc)
        sums = np.zeros((nlist, xq.shape[1]), dtype=np.int64)
        np.add.at(sums, lab, xq.astype(np.int64))
        cnt = np.bincount(lab, minlength=nlist)
        amax = np.abs(sums).max(axis=1)
        upd = (cnt > 0) & (amax > 0)
        sc = _F(127) / amax[upd].astype(np.float32)
        qc[upd] = np.rint(sums[upd].astype(np.float32) * sc[:, None]).clip(-127, 127).astype(np.int8)
    return qc, centroid_factor(qc)


def build_lists(labels: np.ndarray, nlist: int):
    """-> (order: row ids in list order, offsets [nlist+1])."""
    order = np.lexsort((np.arange(len(labels)), labels)).astype(np.int64)
    counts = np.bincount(labels, minlength=nlist)
    off = np.zeros(nlist + 1, dtype=np.int64)
    off[1:] = np.cumsum(counts)
    return order, off


def probes(qq: np.ndarray, qc: np.ndarray, fc: np.ndarray, nprobe: int) -> np.ndarray:
    s = coarse_scores(qq, qc, fc)
    ids = np.broadcast_to(np.arange(qc.shape[0]), s.shape)
    order = np.lexsort((ids, -s), axis=1)[:, :nprobe]
    return order.astype(np.int64)


def search(qq, qinv, codes, inv, labels, qc, fc, nprobe: int, k: int, probe_ids=None):
    """Exact IVF-Flat int8 search.  codes/inv/labels: per row (original row order).
    probe_ids: optional [nq][nprobe] lists to scan (default: computed from qc/fc).
    Returns (scores f32 [nq][k], rows int64 [nq][k])."""
    nq = qq.shape[0]
    pr = probes(qq, qc, fc, nprobe) if probe_ids is None else np.asarray(probe_ids)
    out_s = np.full((nq, k), -np.inf, dtype=np.float32)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    for i in range(nq):
        rows = np.flatnonzero(np.isin(labels, pr[i]))
        if len(rows) == 0:
            continue
        d = int_dot(qq[i:i + 1], codes[rows])[0].astype(np.float32)
        s = d * (inv[rows] * qinv[i]).astype(np.float32)
        o = np.lexsort((rows, -s))[:k]
        out_s[i, :len(o)] = s[o]
        out_r[i, :len(o)] = rows[o]
    return out_s, out_r


def rerank(cand_rows: np.ndarray, q64: np.ndarray, rows64: np.ndarray, k: int):
    """Exact re-rank of IVF candidates [nq][kc] (rows, -1 = padding) against the original rows:
    f64 dot, then top-k by (score desc, row asc), padded (-inf, -1)."""
    nq = cand_rows.shape[0]
    out_s = np.full((nq, k), -np.inf)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    for i in range(nq):
        rr = cand_rows[i][cand_rows[i] >= 0]
        if len(rr) == 0:
            continue
        sc = rows64[rr] @ q64[i]
        o = np.lexsort((rr, -sc))[:k]
        out_s[i, :len(o)] = sc[o]
        out_r[i, :len(o)] = rr[o]
    return out_s, out_r


# ---- clustered synthetic corpus (k_ivf.hip synth_clustered_kernel) ------------------------------
C_KEY = 1 << 63   # key space of cluster centres
L_KEY = 1 << 62   # key space of the row -> cluster draw


def clustered_raw(cseed: int, ncenters: int, seed: int, row0: int, n: int, dim: int) -> np.ndarray:
    """int64 [n][dim]: centre(cluster(r)) + noise(r), both synth.raw_rows-style odd integers;
    cluster(r) = (splitmix64(bn + L_KEY + r) >> 32) % ncenters, bn = splitmix64(seed)."""
    bn = synth.splitmix64_int(seed)
    rows = np.arange(row0, row0 + n, dtype=np.uint64)
    lab = ((synth.splitmix64(np.uint64(bn) + np.uint64(L_KEY) + rows) >> np.uint64(32))
           % np.uint64(ncenters)).astype(np.int64)
    bc = np.uint64(synth.splitmix64_int(cseed))
    ckey = np.uint64(C_KEY) + lab.astype(np.uint64)[:, None] * np.uint64(dim) + np.arange(dim, dtype=np.uint64)[None, :]
    centre = 2 * (synth.splitmix64(bc + ckey) >> np.uint64(40)).astype(np.int64) + 1 - (1 << 24)
    noise = synth.raw_rows(seed, row0, n, dim)
    return centre + noise


def clustered_rows(cseed, ncenters, seed, row0, n, dim, dtype="f32"):
    x = synth.normalize_exact(clustered_raw(cseed, ncenters, seed, row0, n, dim))
    if dtype == "f32":
        return x
    if dtype == "bf16":
        return synth.f32_to_bf16_bits(x)
    if dtype == "f16":
        return x.astype(np.float16)
    raise ValueError(dtype)
