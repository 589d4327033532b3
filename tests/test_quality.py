"""CPU: retrieval quality metrics (rfx.quality) — recall@k and the citation recall that extends the
reference benchmark's citation_hit (scripts/benchmark/metrics.py:73-92, same matching rule)."""
import pytest

from rfx.quality import citation_recall_at_k, recall_at_k


def test_citation_recall_matches_citation_hit_rule():
    cites = [{"sourceId": "DOC-1"}, {"title": "doc-3"}, {"uri": "x"}, {"doc_id": "doc-2"}]
    assert citation_recall_at_k(cites, [], 5) is None
    assert citation_recall_at_k(cites, ["doc-1"], 1) == 1.0
    assert citation_recall_at_k(cites, ["doc-1", "doc-2"], 3) == 0.5   # doc-2 is 4th
    assert citation_recall_at_k(cites, ["doc-1", "doc-2"], 4) == 1.0
    assert citation_recall_at_k([], ["a"], 3) == 0.0


def test_recall_at_k():
    truth = [[1, 2, 3], [4, 5, -1], [-1, -1, -1]]
    assert recall_at_k([[3, 2, 1], [5, 9, 9], [7, 8, 9]], truth, 3) == pytest.approx((1.0 + 0.5) / 2)
    assert recall_at_k([[1, 9, 9]], [[1, 2, 3]], 1) == 1.0
    with pytest.raises(ValueError):
        recall_at_k([[1]], [[1], [2]], 1)


def test_citation_recall_reference_rule_pinned_by_reference_outputs(golden_dir):
    """rule="reference" agrees with the reference's own citation_hit on every captured case
    (tests/golden/ref_citation_hit.json, outputs of scripts/benchmark/metrics.py)."""
    import json
    import os

    cases = json.load(open(os.path.join(golden_dir, "ref_citation_hit.json")))["cases"]
    for c in cases:
        r = citation_recall_at_k(c["citations"], c["gold"], len(c["citations"]) or 1, rule="reference")
        if c["citation_hit"] is None:
            assert r is None
        else:
            assert (r > 0) == (c["citation_hit"] == 1), c


def test_harness_flow_counts_documents_with_rule_any(golden_dir):
    """The benchmark harness flow end to end on the CPU: adapter response -> chat route payloads
    (chat.py:576-586 restated) -> SSE frames -> the harness's parse (run_benchmark.py:196-216
    restated) -> recall.  The reference rule sees only "cit-<i>"; rule="any" counts the document."""
    import os

    from fakes import OracleRetriever
    from oracle import mock_ref
    from rfx.adapter import LocalGpuRag

    rag = LocalGpuRag(OracleRetriever(), top_k=5)
    st = rag.create_store("bench")
    rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md",
                    chunking_config={"white_space_config": {"max_tokens_per_chunk": 3, "max_overlap_tokens": 0}})
    resp = rag.ask(contents="What does the mock-mode assistant do?", store_names=[st], metadata_filter=None, model="m")
    frames = mock_ref.citation_frames(rag.extract_citations_from_response(resp)) + ["data: [DONE]\n\n"]
    cites = mock_ref.harness_citations(frames)
    assert len(cites) == 5 and cites[0]["sourceId"] == "cit-0"
    assert citation_recall_at_k(cites, ["sample-report.md"], 5, rule="reference") == 0.0
    assert citation_recall_at_k(cites, ["sample-report.md"], 5, rule="any") == 1.0
    assert citation_recall_at_k(cites, ["sample-report.md", "missing.md"], 5, rule="any") == 0.5
