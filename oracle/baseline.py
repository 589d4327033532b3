"""CPU baseline timing (bench.py cpu_baseline leg): the oracle's brute-force top-k on a bounded
sample of the benchmark corpus, on the host cores.  Rows are widened block by block."""
import time

import numpy as np

from . import search, synth


def time_topk(rows_stored: np.ndarray, dtype: str, queries64: np.ndarray, k: int, block: int = 65536):
    """Seconds to compute the exact top-k of all queries over rows_stored (row-blocked)."""
    t0 = time.perf_counter()
    nq = queries64.shape[0]
    best_s = np.full((nq, k), -np.inf)
    best_r = np.full((nq, k), -1, dtype=np.int64)
    q32 = queries64.astype(np.float32)
    for b in range(0, rows_stored.shape[0], block):
        blk = synth.to_f64(rows_stored[b:b + block], dtype).astype(np.float32)
        s = (q32 @ blk.T).astype(np.float64)
        m = min(k, s.shape[1])
        part = np.argpartition(-s, m - 1, axis=1)[:, :m]
        ps = np.take_along_axis(s, part, axis=1)
        cs = np.concatenate([best_s, ps], axis=1)
        cr = np.concatenate([best_r, part + b], axis=1)
        order = np.lexsort((cr, -cs), axis=1)[:, :k]
        best_s = np.take_along_axis(cs, order, axis=1)
        best_r = np.take_along_axis(cr, order, axis=1)
    return time.perf_counter() - t0, best_s, best_r


def time_mock_plumbing(n: int = 20000):
    """µs per call of the reference mock retriever's response build + citation extraction
    (restated in oracle.mock_ref: gemini_rag.py:673-718, 554-595)."""
    from . import mock_ref
    q = "What is the purpose of the /api/chat endpoint in this service?"
    t0 = time.perf_counter()
    for _ in range(n):
        mock_ref.extract_citations(mock_ref.mock_response(q, ["fileSearchStores/x"]))
    return (time.perf_counter() - t0) / n * 1e6
