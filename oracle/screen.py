"""Oracle restatement of the exact two-pass scan (kernel 10, csrc/k_scan_screen.h + k_screen.hip;
DESIGN.md §4.10).  TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's checks, never by the product path.

The reference has no counterpart (its retrieval arithmetic runs inside Google's File Search,
backend/app/services/gemini_rag.py:517-551); the two-pass scan must return exactly what the
brute-force rule of oracle/search.py returns (score desc, row asc), so the pinned quantity is
search.topk itself.  This module restates the int8 copy bit-for-bit (codes, tile scales, live
words; stats to f64 rounding) and the screen's selection rule, so a test can show on the CPU that
the rule keeps every row of the true top-k.

Quantiser (per 32-row tile; dead rows = any NaN element: code 0, live bit clear):
    s_t = f32(amax over live rows) / 127 (IEEE f32 division; 0 when the tile has no live row)
    c   = clamp(rint(f32(x) / s_t), -127, 127)
    stats = (max ||x||, max ||x - s_t c||) over live rows, rounded up to f32, and max s_t (the
            screen kernel's fast-path bound: no per-tile data on the fast path).
Queries: s_y, c_y likewise per query; E_q = Xmax ||y - s_y c_y|| + Emax ||s_y c_y|| (Cauchy-Schwarz);
    e2 = (2 E_q + 4e-7 (Xmax + Emax) ||s_y c_y|| + 2.4e-7 Xmax (||s_y c_y|| + ||y - s_y c_y||)) (1 + 1e-5) / s_y,
    rounded up to f32 (the 2.4e-7 term: two f32 ulps of the k-th exact score, so a row whose exact
    score rounds to the k-th's f32 with a smaller row id survives under the score rule).
Screen score (units of s_y): A = f32(c_x . c_y) * s_t (one f32 rounding).  Survivors of a query:
rows with A >= a_k - e2 (a_k = k-th best A over live rows); exact re-score; top-k.
"""
import numpy as np

TM = 32


def _f32_up(v):
    v = np.asarray(v, dtype=np.float64)
    f = v.astype(np.float32)
    lo = f.astype(np.float64) < v
    f[lo] = np.nextafter(f[lo], np.float32(np.inf))
    return f


def quantize_tiles(rows32):
    """rows32: [n][D] f32 (the stored values widened exactly; NaN rows dead), n a multiple of 32
    or not (padded with dead rows).  Returns (codes int8 [ntiles*32][D], scales f32 [ntiles],
    live uint32 [ntiles], stats f32 [2])."""
    x = np.asarray(rows32, dtype=np.float32)
    n, d = x.shape
    nt = -(-n // TM)
    pad = np.full((nt * TM - n, d), np.nan, dtype=np.float32)
    x = np.concatenate([x, pad]) if len(pad) else x
    dead = np.isnan(x).any(axis=1)
    xl = np.where(dead[:, None], np.float32(0), x).reshape(nt, TM, d)
    amax = np.abs(xl).max(axis=(1, 2)).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.where(amax > 0, amax / np.float32(127), np.float32(0)).astype(np.float32)
        q = np.rint(xl / s[:, None, None]).astype(np.float32)
    q = np.where(s[:, None, None] > 0, q, np.float32(0))
    c = np.clip(q, -127, 127).astype(np.int8).reshape(nt * TM, d)
    c[dead] = 0
    live = np.zeros(nt, dtype=np.uint32)
    for t in range(nt):
        bits = ~dead[t * TM:(t + 1) * TM]
        live[t] = np.uint32(sum(1 << i for i in range(TM) if bits[i]))
    xd = x.astype(np.float64)
    rec = np.repeat(s.astype(np.float64), TM)[:, None] * c.astype(np.float64)
    xn = np.sqrt((np.where(dead[:, None], 0.0, xd) ** 2).sum(axis=1))
    en = np.sqrt((np.where(dead[:, None], 0.0, xd - rec) ** 2).sum(axis=1))
    stats = np.array([_f32_up(xn[~dead].max()) if (~dead).any() else 0.0,
                      _f32_up(en[~dead].max()) if (~dead).any() else 0.0,
                      s.max() if s.size else 0.0], dtype=np.float32)
    return c, s, live, stats


def quantize_queries(q32, stats):
    """q32 [nq][D] f32 (widened stored queries) -> (codes int8 [nq][D], e2 f32 [nq], s f32 [nq]);
    stats as quantize_tiles returns them (the first two are used)."""
    y = np.asarray(q32, dtype=np.float32)
    amax = np.abs(y).max(axis=1).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.where(amax > 0, amax / np.float32(127), np.float32(0)).astype(np.float32)
        q = np.rint(y / s[:, None]).astype(np.float32)
    q = np.where(s[:, None] > 0, q, np.float32(0))
    c = np.clip(q, -127, 127).astype(np.int8)
    yd = y.astype(np.float64)
    rec = s.astype(np.float64)[:, None] * c.astype(np.float64)
    ey = np.sqrt(((yd - rec) ** 2).sum(axis=1))
    yh = s.astype(np.float64) * np.sqrt((c.astype(np.int64) ** 2).sum(axis=1).astype(np.float64))
    xm, em = float(stats[0]), float(stats[1])
    eq = xm * ey + em * yh
    with np.errstate(divide="ignore", invalid="ignore"):
        e2 = np.where(s > 0, (2.0 * eq + 4e-7 * (xm + em) * yh + 2.4e-7 * xm * (yh + ey)) * (1.0 + 1e-5)
                      / s.astype(np.float64), 0.0)
    return c, _f32_up(e2), s


def screen_scores(codes, scales, qcodes):
    """A [nq][n] (f32): i32 dot of the codes times the tile scale, one f32 rounding."""
    dots = qcodes.astype(np.float32) @ codes.astype(np.float32).T  # |dot| < 2^24: exact in f32
    tile_s = np.repeat(scales, TM)[: codes.shape[0]]
    return (dots * tile_s[None, :]).astype(np.float32)


def screen_topk(q32, rows32, k):
    """The two-pass rule end to end on the CPU.  Returns (scores f64 [nq][k], rows [nq][k],
    survivors [nq]) — equal to search.topk(q, rows, k) whenever the bound is rigorous."""
    x = np.asarray(rows32, dtype=np.float32)
    n = x.shape[0]
    codes, scales, live, stats = quantize_tiles(x)
    qc, e2, _ = quantize_queries(q32, stats)
    A = screen_scores(codes, scales, qc)[:, :n]
    dead = np.isnan(x).any(axis=1)
    A[:, dead] = -np.inf
    nq = A.shape[0]
    out_s = np.full((nq, k), -np.inf)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    nsv = np.zeros(nq, dtype=np.int64)
    q64 = np.asarray(q32, dtype=np.float64)
    for i in range(nq):
        a = A[i]
        nlive = int((~dead).sum())
        if nlive >= k:
            ak = np.partition(a[~dead], nlive - k)[nlive - k]
            t = np.float32(ak - e2[i])
        else:
            t = -np.inf
        sv = np.nonzero((a >= t) & ~dead)[0]
        nsv[i] = sv.size
        ex = x[sv].astype(np.float64) @ q64[i]
        o = np.lexsort((sv, -ex))[:k]
        out_s[i, :o.size] = ex[o]
        out_r[i, :o.size] = sv[o]
    return out_s, out_r, nsv
