"""CPU: the oracle against the reference's own golden vectors and against its committed fixtures."""
import json
import os

import numpy as np
import pytest

from oracle import embed, mock_ref, search, synth, textproc


def test_normalize_matches_reference(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "ref_normalize.json"), encoding="utf-8"))
    assert len(d["cases"]) >= 30
    for c in d["cases"]:
        assert textproc.normalize(c["input"]) == c["normalized"], c["input"]


def test_byte_tokenizer_equals_reference_normalize(golden_dir):
    """The byte-level tokeniser used by the index (after str.lower()) == reference _normalize."""
    d = json.load(open(os.path.join(golden_dir, "ref_normalize.json"), encoding="utf-8"))
    for c in d["cases"]:
        toks = textproc.tokens_bytes(c["input"].lower().encode("utf-8"))
        assert " ".join(t.decode() for t in toks) == c["normalized"], c["input"]


@pytest.mark.parametrize("contents,expected", [
    ("plain", "plain"),
    ([{"role": "user", "parts": [{"text": "first"}]}, {"role": "user", "parts": [{"text": " last "}]}], "last"),
    ([{"role": "user", "parts": [{"text": "q"}]}, {"role": "model", "parts": [{"text": "  "}]}], "q"),
    (["a string", {"parts": []}], "a string"),
    ([], "[]"),
])
def test_contents_to_text(contents, expected):
    assert textproc.contents_to_text(contents) == expected


def test_mock_structure():
    """gemini_rag.py:704-718 + 554-595: one rank-0 citation with the fixed mock fields."""
    q = "What is RAG?" * 20
    cits = mock_ref.extract_citations(mock_ref.mock_response(q, ["fileSearchStores/s1"]))
    assert cits == [{"index": 0, "source_type": "retrieved_context", "uri": "mock://document",
                     "title": "Mock Document", "snippet": "Mock snippet: " + q[:128], "store": "fileSearchStores/s1"}]
    assert mock_ref.extract_citations(mock_ref.mock_response("x", []))[0]["store"] == "store/mock"
    assert mock_ref.first_stream_text("") == "[mock-mode] response"


def test_chunker_cfg1(golden_dir):
    raw = open(os.path.join(golden_dir, "sample_report.md"), "rb").read()
    spans = textproc.chunk_whitespace(raw, 3, 0)
    assert len(spans) == 32  # BASELINE config 1: "~32 chunks"
    assert raw[spans[0][0]:spans[0][1]] == b"# Demo Source"
    # overlapping windows share exactly `overlap` tokens
    sp = textproc.chunk_whitespace(raw, 10, 3)
    toks = raw.split()
    assert raw[sp[1][0]:sp[1][1]].split()[:3] == toks[7:10]


def test_chunker_edges():
    assert textproc.chunk_whitespace(b"", 5, 0) == []
    assert textproc.chunk_whitespace(b"   \n\t ", 5, 0) == []
    assert textproc.chunk_whitespace(b"one", 5, 2) == [(0, 3)]
    with pytest.raises(ValueError):
        textproc.chunk_whitespace(b"x", 3, 3)


def test_cfg1_fixture_reproduces(golden_dir):
    """The committed config-1 fixture is what the oracle computes today."""
    fx = json.load(open(os.path.join(golden_dir, "cfg1_sample_report.json")))
    raw = open(os.path.join(golden_dir, "sample_report.md"), "rb").read()
    spans = textproc.chunk_whitespace(raw, 3, 0)
    wt = embed.weights_int(fx["V"], fx["dim"], 0x5241475F454D4244)
    X = embed.embed(*textproc.featurize(raw, spans, fx["V"], 0x5241475F544F4B4E), fx["V"], wt).astype(np.float64)
    for case in fx["queries"]:
        qb = case["question"].lower().encode()
        Q = embed.embed(*textproc.featurize(qb, [(0, len(qb))], fx["V"], 0x5241475F544F4B4E), fx["V"], wt).astype(np.float64)
        s, r = search.topk(Q, X, fx["k"])
        assert r[0][r[0] >= 0].tolist() == case["rows"]
        assert np.allclose(s[0][r[0] >= 0], case["scores"], rtol=0, atol=1e-12)


def test_synth_fixture(golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_small.npz"))
    for dt in ("f32", "bf16", "f16"):
        assert synth.synth_rows(3, 1000, 4, 768, dt).tobytes() == z[dt].tobytes()
    X = synth.to_f64(synth.synth_rows(7, 0, 3000, 768, "f32"), "f32")
    Q = synth.to_f64(synth.synth_rows(8, 0, 4, 768, "f32"), "f32")
    s, r = search.topk(Q, X, 10, row_block=777)
    assert (r == z["top_r"]).all() and np.array_equal(s, z["top_s"])


def test_synth_rows_are_unit_norm():
    x = synth.synth_rows(0, 0, 50, 768, "f32").astype(np.float64)
    assert np.allclose(np.linalg.norm(x, axis=1), 1.0, atol=1e-6)
    raw = synth.raw_rows(0, 0, 10, 64)
    assert (raw % 2 == 1).all() and (np.abs(raw) < 2 ** 24).all()


def test_bf16_rounding_rule():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.5, np.inf, 3.0e-39], dtype=np.float32)
    b = synth.f32_to_bf16_bits(x)
    # 1.00390625 is the exact midpoint between bf16 1.0 and 1.0078125 -> ties to even (1.0)
    assert b[1] == 0x3F80 and b[2] == 0x3F82
    assert synth.bf16_bits_to_f32(b)[3] == -2.5 and np.isinf(synth.bf16_bits_to_f32(b)[4])
    nan = synth.f32_to_bf16_bits(np.array([np.nan], dtype=np.float32))
    assert np.isnan(synth.bf16_bits_to_f32(nan))[0]


def test_topk_tie_rule_and_padding():
    X = np.array([[1.0, 0], [0, 1.0], [1.0, 0], [0.5, 0.5], [np.nan, 0]])
    Q = np.array([[1.0, 0.0]])
    s, r = search.topk(Q, X, 6)
    assert r[0].tolist() == [0, 2, 3, 1, -1, -1]  # equal scores: lower row first; NaN row excluded
    assert np.isneginf(s[0][4:]).all()


def test_check_topk_tie_band():
    ref_s = np.array([[0.5, 0.4, 0.3]])
    ref_r = np.array([[1, 2, 3]])
    sc = {1: 0.5, 2: 0.4, 3: 0.3, 4: 0.3 - 1e-7, 5: 0.2}
    f = lambda q, rows: np.array([sc[int(x)] for x in rows])
    assert search.check_topk(ref_s, ref_r, ref_s, ref_r, f) == []
    # near-tie swap across the boundary is accepted, a real miss is not
    assert search.check_topk(np.array([[0.5, 0.4, 0.3 - 1e-7]]), np.array([[1, 2, 4]]), ref_s, ref_r, f) == []
    assert search.check_topk(np.array([[0.5, 0.4, 0.2]]), np.array([[1, 2, 5]]), ref_s, ref_r, f) != []


def test_check_topk_rejects_duplicate_rows():
    """[a, a, c] against [a, b, c] with |s_a - s_b| inside the tie band must fail."""
    ref_s = np.array([[0.5, 0.5 - 1e-7, 0.3]])
    ref_r = np.array([[1, 2, 3]])
    sc = {1: 0.5, 2: 0.5 - 1e-7, 3: 0.3}
    f = lambda q, rows: np.array([sc[int(x)] for x in rows])
    probs = search.check_topk(np.array([[0.5, 0.5, 0.3]]), np.array([[1, 1, 3]]), ref_s, ref_r, f)
    assert probs and "duplicate" in probs[0]
    # the legal near-tie swap of the same two rows still passes
    assert search.check_topk(np.array([[0.5 - 1e-7, 0.5, 0.3]]), np.array([[2, 1, 3]]), ref_s, ref_r, f) == []


def test_check_topk_requires_rows_above_band():
    """A row scoring above the k-th score's band must be returned even if the GPU list is
    otherwise ordered and within tolerance."""
    ref_s = np.array([[0.9, 0.5, 0.5 - 1e-7]])
    ref_r = np.array([[7, 1, 2]])
    sc = {7: 0.9, 1: 0.5, 2: 0.5 - 1e-7, 3: 0.5 - 1.5e-6}
    f = lambda q, rows: np.array([sc[int(x)] for x in rows])
    # row 7 (0.9) replaced by two near-ties of the k-th score: must fail
    probs = search.check_topk(np.array([[0.5, 0.5 - 1e-7, 0.5 - 1.5e-6]]), np.array([[1, 2, 3]]), ref_s, ref_r, f)
    assert any("missing" in p or "below" in p or "differ" in p for p in probs)


def test_embed_exactness_bound():
    """|e| stays below 2^24 quanta for the maximum chunk (65536 tokens), so f32 MFMA accumulation
    is exact in any order (k_embed.hip)."""
    assert textproc.MAX_TOKENS_PER_CHUNK * 127 < 2 ** 24
    wt = embed.weights_int(64, 32, 1)
    assert wt.min() >= -127 and wt.max() <= 127
    # w=(u>>32)*255>>32 - 127 covers the full range
    big = embed.weights_int(4096, 64, 2)
    assert big.min() == -127 and big.max() == 127
