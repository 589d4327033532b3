"""Brute-force inner-product top-k (oracle restatement of the scan + merge kernels).

Ranking rule: score descending, then row id ascending.  Scores are
accumulated in float64 over the exactly-widened stored values.  Rows whose stored vector
contains NaN (tombstones) are never returned; results are padded with (-inf, -1).
"""
import math

import numpy as np


def topk(queries64: np.ndarray, rows64: np.ndarray, k: int, row_block: int = 1 << 18):
    """Return (scores f64 [nq][k], rows int64 [nq][k]) for float64 inputs."""
    queries64 = np.asarray(queries64, dtype=np.float64)
    nq = queries64.shape[0]
    best_s = np.full((nq, 0), -np.inf)
    best_r = np.zeros((nq, 0), dtype=np.int64)
    n = rows64.shape[0]
    for b in range(0, n, row_block):
        blk = np.asarray(rows64[b:b + row_block], dtype=np.float64)
        dead = np.isnan(blk).any(axis=1)
        s = queries64 @ np.where(dead[:, None], 0.0, blk).T     # [nq][B]
        s[:, dead] = -np.inf
        rows = np.arange(b, b + blk.shape[0], dtype=np.int64)
        m = min(k, s.shape[1])
        part = np.argpartition(-s, m - 1, axis=1)[:, :m]
        kth = np.take_along_axis(s, part, axis=1).min(axis=1, keepdims=True)
        keep = (s >= kth) & ~dead[None, :]
        cnt = keep.sum(axis=1)
        width = int(cnt.max()) + best_s.shape[1] if nq else 0
        cs = np.full((nq, width), -np.inf)
        cr = np.full((nq, width), np.iinfo(np.int64).max, dtype=np.int64)
        for i in range(nq):
            ks = s[i][keep[i]]
            kr = rows[keep[i]]
            allr = np.concatenate([best_r[i], kr])
            alls = np.concatenate([best_s[i], ks])
            cs[i, :len(alls)] = alls
            cr[i, :len(allr)] = allr
        order = np.lexsort((cr, -cs), axis=1)[:, :k]
        best_s = np.take_along_axis(cs, order, axis=1)
        best_r = np.take_along_axis(cr, order, axis=1)
        best_r[best_r == np.iinfo(np.int64).max] = -1
        best_r[best_r < 0] = -1
        best_s[best_r < 0] = -np.inf
        # drop padding so the next merge sees only real candidates
        width = int((best_r >= 0).sum(axis=1).max()) if nq else 0
        best_s, best_r = best_s[:, :width], best_r[:, :width]
        best_r = np.where(best_r < 0, np.iinfo(np.int64).max, best_r)
    out_s = np.full((nq, k), -np.inf)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    w = min(k, best_s.shape[1])
    out_s[:, :w] = best_s[:, :w]
    out_r[:, :w] = np.where(best_r[:, :w] == np.iinfo(np.int64).max, -1, best_r[:, :w])
    out_s[out_r < 0] = -np.inf
    return out_s, out_r


def _merge_best(best_s, best_r, cand_s, cand_r, k):
    """Top-k (score desc, row asc) of two candidate lists of one query."""
    s = np.concatenate([best_s, cand_s])
    r = np.concatenate([best_r, cand_r])
    o = np.lexsort((r, -s))[:k]
    return s[o], r[o]


def topk_blocks(queries64: np.ndarray, blocks, k: int, first_rows: int = 1 << 16):
    """Exact top-k over a corpus delivered block by block, for corpora too large to widen to f64
    at once (BASELINE configs 3/4: 10M x 768, 12.5M x 1024).  Same result as topk() over the
    concatenated rows, including the tie rule (score desc, row asc) and NaN-row exclusion.

    blocks: iterable of (row0, rows_f32) where rows_f32 [B][d] are the STORED values widened
    exactly to f32 (f32, bf16 and f16 all widen exactly); queries64 must be exactly
    representable in f32 (they are widened stored queries).

    Two stages per block:
      1. screen: S = rows_f32 @ q_f32 in f32 (BLAS).  For any summation order the rounding error
         of a d-term f32 dot is <= gamma_d * sum|x_i q_i| <= gamma_d * sqrt(d) * max|x| * ||q||_2
         = eb (gamma_d = d u / (1 - d u), u = 2^-24).  A row whose exact score is >= the exact
         k-th best score E_k of the block has S >= E_k - eb >= F_k - 2 eb, where F_k is the k-th
         best screened score (order statistics move by at most eb); F_k is bounded below by the
         k-th best of the block's first `first_rows` rows, and rows below the running global
         k-th best (exact) minus eb cannot enter the result either.
      2. rescore the survivors (exact products, one rounding of their sum) and merge with the
         running top-k.
    """
    q64 = np.asarray(queries64, dtype=np.float64)
    q32 = q64.astype(np.float32)
    if not np.array_equal(q32.astype(np.float64), q64):
        raise ValueError("queries must be exactly representable in f32")
    nq, d = q64.shape
    u = 2.0 ** -24
    gam = d * u / (1.0 - d * u)
    qn = np.sqrt((q64 * q64).sum(axis=1))
    best = [(np.zeros(0), np.zeros(0, dtype=np.int64)) for _ in range(nq)]
    for row0, X in blocks:
        X = np.ascontiguousarray(X, dtype=np.float32)
        B = X.shape[0]
        if B == 0:
            continue
        S = q32 @ X.T  # [nq][B], f32
        dead = np.isnan(S)
        S[dead] = -np.inf
        amax = float(np.max(np.abs(X), where=~np.isnan(X), initial=0.0))
        eb = gam * np.sqrt(d) * amax * qn * 1.001 + 1e-30  # [nq]
        m = min(k, B, first_rows)
        head = S[:, :min(B, first_rows)]
        fk = -np.partition(-head, m - 1, axis=1)[:, m - 1] if m >= 1 else np.full(nq, -np.inf)
        thr = fk - 2.0 * eb
        for i in range(nq):
            if len(best[i][0]) >= k:
                thr[i] = max(thr[i], best[i][0][k - 1] - eb[i])
        keep = (S >= thr[:, None]) & ~dead
        for i in range(nq):
            c = np.nonzero(keep[i])[0]
            if c.size == 0:
                continue
            # products of f32-representable values are exact in f64; fsum rounds their sum once,
            # so equal rows score equal (exact ties stay ties, whatever the summation order)
            ex = np.array([math.fsum(v) for v in X[c].astype(np.float64) * q64[i]])
            best[i] = _merge_best(best[i][0], best[i][1], ex, c.astype(np.int64) + row0, k)
    out_s = np.full((nq, k), -np.inf)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    for i, (s, r) in enumerate(best):
        out_s[i, :len(s)] = s
        out_r[i, :len(r)] = r
    return out_s, out_r


def check_topk(gpu_s, gpu_r, ref_s, ref_r, scores_of, tol=1e-5, tie_band=2e-6):
    """Parity rule.  Row lists must be identical, except that two rows whose
    reference scores differ by <= tie_band may appear in either order and may swap across the
    k-th boundary.  GPU scores must be within `tol` of the reference fp64 score of the SAME row.
    `scores_of(q, rows)` returns reference fp64 scores for arbitrary rows of query q.
    Returns a list of human-readable problems (empty = pass)."""
    problems = []
    nq, k = ref_r.shape
    for q in range(nq):
        g, r = gpu_r[q], ref_r[q]
        gl = g[g >= 0]
        if np.unique(gl).size != gl.size:
            # a merge that emits one row twice must never pass, tie band or not
            problems.append(f"q{q}: duplicate rows returned {g.tolist()}")
            continue
        if np.array_equal(g, r):
            live = g >= 0
            if live.any():
                d = np.abs(gpu_s[q][live].astype(np.float64) - ref_s[q][live])
                if d.max() > tol:
                    problems.append(f"q{q}: score err {d.max():.3g} > {tol}")
            continue
        if (g < 0).sum() != (r < 0).sum():
            problems.append(f"q{q}: live count differs {g.tolist()} vs {r.tolist()}")
            continue
        live = g >= 0
        sg = scores_of(q, g[live])
        d = np.abs(gpu_s[q][live].astype(np.float64) - sg)
        if d.max() > tol:
            problems.append(f"q{q}: score err {d.max():.3g} > {tol}")
        kth = ref_s[q][live.sum() - 1]
        if (sg < kth - tie_band).any():
            problems.append(f"q{q}: returned row below k-th score band: {g.tolist()} vs {r.tolist()}")
        # the returned set equals the reference set outside the band: every reference row scoring
        # above the k-th score's band must be returned
        rl = r[r >= 0]
        must = rl[ref_s[q][r >= 0] > kth + tie_band]
        missing = np.setdiff1d(must, gl)
        if missing.size:
            problems.append(f"q{q}: rows {missing.tolist()} above the tie band are missing: {g.tolist()} vs {r.tolist()}")
        # order: GPU order must be non-increasing in reference score up to the tie band
        if (np.diff(sg) > tie_band).any():
            problems.append(f"q{q}: order violates ranking beyond tie band")
        # any mismatched position must be explained by a near-tie
        for a, b in zip(g[live], r[live]):
            if a != b:
                sa = scores_of(q, np.array([a]))[0]
                sb = scores_of(q, np.array([b]))[0]
                if abs(sa - sb) > tie_band:
                    problems.append(f"q{q}: row {a} vs {b} differ by {abs(sa - sb):.3g} (> tie band)")
                    break
    return problems
