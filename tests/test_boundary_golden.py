"""CPU: the drop-in boundary against the reference's OWN test vectors (tests/golden/ref_boundary.json,
extracted from backend/tests/test_gemini_rag.py and test_chat_stream_helpers.py by
tests/golden/make_ref_boundary.py): LocalGpuRag.extract_citations_from_response and
new_stream_ids satisfy the reference's assertions, and the oracle's restatement of the chat
route's SSE payload builders (chat.py:576-603) reproduces the reference's expected payloads."""
import json
import os
from types import SimpleNamespace

import pytest

from oracle import mock_ref
from rfx.adapter import LocalGpuRag


@pytest.fixture(scope="module")
def gold(golden_dir):
    return json.load(open(os.path.join(golden_dir, "ref_boundary.json")))


def _response(chunks):
    return SimpleNamespace(candidates=[SimpleNamespace(grounding_metadata=SimpleNamespace(grounding_chunks=chunks))])


def _dig(obj, path):
    for p in path:
        obj = obj[p]
    return obj


def test_extract_citations_reference_vector(gold):
    g = gold["extract_citations_valid"]
    ch = g["grounding_chunk"]
    chunk = SimpleNamespace(retrieved_context=SimpleNamespace(**ch["retrieved_context"]), web=ch["web"])
    for impl in (LocalGpuRag.extract_citations_from_response, mock_ref.extract_citations):
        env = {"citations": impl(_response([chunk]))}
        for a in g["asserts"]:
            if "len_of" in a:
                assert len(env[a["len_of"]]) == a["equals"], a
            else:
                assert _dig(env[a["path"][0]], a["path"][1:]) == a["equals"], a


def test_extract_citations_empty_reference_cases(gold):
    assert gold["extract_citations_empty"]["expect"] == []
    cases = [SimpleNamespace(candidates=[]),
             SimpleNamespace(candidates=[SimpleNamespace(grounding_metadata=None)]),
             SimpleNamespace(candidates=[SimpleNamespace(grounding_metadata=SimpleNamespace(grounding_chunks=None))]),
             SimpleNamespace()]  # no candidates attribute at all (test_gemini_rag.py:74-83)
    for resp in cases:
        assert LocalGpuRag.extract_citations_from_response(resp) == []


def test_stream_ids_reference_contract(gold):
    a, b = LocalGpuRag.new_stream_ids()
    assert isinstance(a, str) and a != b and [len(a), len(b)] == gold["stream_ids"]["length"] * 2


def test_citation_frame_restatement_matches_reference_vector(gold):
    g = gold["citation_frame"]
    assert mock_ref.citation_frame_payloads([g["citation"]]) == [g["payload"]]
    frame = mock_ref.citation_frames([g["citation"]])[0]
    assert frame.startswith("data: ") and frame.endswith("\n\n")
    assert json.loads(frame[len("data: "):].strip()) == g["payload"]


def test_finish_frame_restatement_matches_reference_vector(gold):
    g = gold["finish_frame"]
    env = {"payload": mock_ref.finish_frame_payload(**g["kwargs"])}
    assert g["asserts"]
    for a in g["asserts"]:
        assert _dig(env[a["path"][0]], a["path"][1:]) == a["equals"], a


def payload_shape_ok(payloads, ref_payload, titles, snippets):
    """The chat route's payloads built from an adapter response have exactly the reference
    payload's keys and fixed values, and sourceId = cit-<rank> (citation index = rank)."""
    assert [p["sourceId"] for p in payloads] == [f"cit-{i}" for i in range(len(payloads))]
    for p, t, s in zip(payloads, titles, snippets):
        assert set(p) == set(ref_payload)
        assert p["type"] == ref_payload["type"] and p["mediaType"] == ref_payload["mediaType"]
        assert p["title"] == t and p["snippet"] == s


@pytest.mark.parametrize("k", [1, 5])
def test_adapter_citations_make_reference_shaped_frames(gold, golden_dir, k):
    from fakes import OracleRetriever

    rag = LocalGpuRag(OracleRetriever(), top_k=k)
    st = rag.create_store("demo")
    rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md",
                    chunking_config={"white_space_config": {"max_tokens_per_chunk": 3, "max_overlap_tokens": 0}})
    q = "How does the mock-mode document assistant cite sources?"
    chunks = list(rag.ask_stream(contents=[{"role": "user", "parts": [{"text": q}]}], store_names=[st],
                                 metadata_filter=None, model="gemini-2.5-flash"))
    cits = rag.extract_citations_from_response(chunks[1])
    assert len(cits) == k
    gc = chunks[1].candidates[0].grounding_metadata.grounding_chunks
    payload_shape_ok(mock_ref.citation_frame_payloads(cits), gold["citation_frame"]["payload"],
                     ["sample-report.md"] * k, [g.retrieved_context.text for g in gc])
