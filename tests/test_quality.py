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
