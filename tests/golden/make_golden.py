"""Generate the oracle's committed numeric fixtures (run in the build container).

  cfg1_sample_report.json  BASELINE config 1: docs/demo/sample-report.md chunked into 3-token
                           whitespace windows (~32 chunks), embedded (dim 768, f32), top-5 per
                           question: expected rows, fp64 scores, snippets.
  synth_small.npz          generator fixture: seed 3 rows 1000..1003 (dim 768) in f32/bf16/f16
                           bits, plus the top-10 of 4 queries (seed 8) over 3000 rows (seed 7).
The GPU tests compare the HIP path against these files AND against the live oracle.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import embed, search, synth, textproc  # noqa: E402

W_SEED, H_SEED, V = 0x5241475F454D4244, 0x5241475F544F4B4E, 4096
QUESTIONS = [
    "What does the demo flow show?",
    "How are uploaded documents ingested?",
    "Do chat answers stream back with source citations?",
    "What replaces Gemini calls in demo mode?",
    "cost and budget visibility",
]


def main():
    text = open(os.path.join(HERE, "sample_report.md"), encoding="utf-8").read()
    qs = QUESTIONS + json.load(open(os.path.join(HERE, "bench_questions.json")))["questions"]
    raw = text.encode()
    spans = textproc.chunk_whitespace(raw, 3, 0)
    chunks = [raw[s:e].decode() for s, e in spans]
    wt = embed.weights_int(V, 768, W_SEED)
    X = embed.embed(*textproc.featurize(raw, spans, V, H_SEED), V, wt, "f32").astype(np.float64)
    qb = [q.lower().encode() for q in qs]
    qraw = b"".join(qb)
    offs = np.cumsum([0] + [len(x) for x in qb])
    Q = embed.embed(*textproc.featurize(qraw, list(zip(offs[:-1], offs[1:])), V, H_SEED), V, wt, "f32").astype(np.float64)
    s, r = search.topk(Q, X, 5)
    out = {"doc": "sample_report.md", "chunking": {"max_tokens_per_chunk": 3, "max_overlap_tokens": 0},
           "n_chunks": len(chunks), "dim": 768, "V": V, "k": 5, "queries": []}
    for i, q in enumerate(qs):
        live = r[i] >= 0
        out["queries"].append({"question": q, "rows": r[i][live].tolist(), "scores": s[i][live].tolist(),
                               "snippets": [chunks[j] for j in r[i][live]]})
    json.dump(out, open(os.path.join(HERE, "cfg1_sample_report.json"), "w"), indent=1)

    rows = {dt: synth.synth_rows(3, 1000, 4, 768, dt) for dt in ("f32", "bf16", "f16")}
    X7 = synth.to_f64(synth.synth_rows(7, 0, 3000, 768, "f32"), "f32")
    Q8 = synth.to_f64(synth.synth_rows(8, 0, 4, 768, "f32"), "f32")
    ts, tr = search.topk(Q8, X7, 10)
    np.savez(os.path.join(HERE, "synth_small.npz"), f32=rows["f32"], bf16=rows["bf16"], f16=rows["f16"],
             top_s=ts, top_r=tr)
    print("n_chunks", len(chunks), "queries", len(qs))


if __name__ == "__main__":
    main()
