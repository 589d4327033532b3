"""Retrieval quality metrics for regression runs ("extend scripts/benchmark
citation_hit (metrics.py:73-92) to recall@k against oracle rows").

citation_recall_at_k reports the FRACTION of gold documents cited within the first k citations
instead of citation_hit's 0/1.  rule="reference" keeps citation_hit's matching exactly (the first
non-empty of doc_id / sourceId / uri / title, case-insensitive; pinned by the reference's own
outputs, tests/golden/ref_citation_hit.json).  Under that rule the harness's citations — parsed
from "source-document" frames as {title, snippet, sourceId} (run_benchmark.py:209-216) — always
match on sourceId "cit-<i>", never on the document, so rule="any" (any of those fields equals a
gold id) is what makes the metric count documents; INTEGRATION.md §5 wires it in.
recall_at_k compares retrieved row ids with the exact (oracle / brute-force) top-k rows.
"""
from typing import Iterable, Optional, Sequence

_FIELDS = ("doc_id", "sourceId", "uri", "title")


def _cite_keys(c: dict, rule: str):
    if rule == "reference":
        return {str(c.get("doc_id") or c.get("sourceId") or c.get("uri") or c.get("title") or "").lower()} - {""}
    if rule == "any":
        return {str(c[f]).lower() for f in _FIELDS if c.get(f)}
    raise ValueError(f"unknown matching rule {rule!r}")


def citation_recall_at_k(citations: Iterable[dict], gold_doc_ids: Sequence[str], k: int,
                         rule: str = "reference") -> Optional[float]:
    """None without gold ids (as citation_hit); else |gold ∩ first-k citations| / |gold|."""
    if not gold_doc_ids:
        return None
    gold = {str(g).lower() for g in gold_doc_ids}
    seen = set()
    for c in list(citations or [])[:k]:
        seen |= _cite_keys(c, rule)
    return len(gold & seen) / len(gold)


def recall_at_k(retrieved: Sequence[Sequence[int]], truth: Sequence[Sequence[int]], k: int) -> float:
    """Mean over queries of |retrieved[:k] ∩ truth[:k]| / |truth[:k]| (rows < 0 = padding, ignored)."""
    if len(retrieved) != len(truth):
        raise ValueError("retrieved and truth must have one row list per query")
    tot, n = 0.0, 0
    for got, ref in zip(retrieved, truth):
        ref_k = {int(r) for r in list(ref)[:k] if int(r) >= 0}
        if not ref_k:
            continue
        got_k = {int(r) for r in list(got)[:k] if int(r) >= 0}
        tot += len(got_k & ref_k) / len(ref_k)
        n += 1
    return tot / n if n else 1.0
