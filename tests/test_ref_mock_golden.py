"""CPU: the reference mock retriever's own outputs pin the restatement and the adapter boundary.

tests/golden/ref_mock.json holds what MockGeminiRag (backend/app/services/gemini_rag.py:602-725)
returned for the fixed question list (tests/golden/bench_questions.json plus edge cases), captured by
importing it in the build container (tests/golden/make_ref_mock.py).  Checked here:
  * oracle.mock_ref.mock_response / first_stream_text / extract_citations reproduce it exactly;
  * the adapter's contents -> question extraction equals the mock's on every case and shape;
  * LocalGpuRag (oracle-backed retriever, top_k = 1) streams the mock's first chunk exactly and a
    second chunk with the mock's attribute structure, citation keys, rank-0 index and store field.
Deliberate difference: with store_names == [] the mock invents one hit on "store/mock"; the local
backend searches no store and returns no hit (tested below)."""
import json
import os

import pytest

from fakes import OracleRetriever
from oracle import mock_ref
from rfx.adapter import LocalGpuRag, contents_to_text


def ns_to_dict(o):
    if isinstance(o, (str, int, float, bool)) or o is None:
        return o
    if isinstance(o, (list, tuple)):
        return [ns_to_dict(x) for x in o]
    if isinstance(o, dict):
        return {k: ns_to_dict(v) for k, v in o.items()}
    return {"__type__": type(o).__name__, **{k: ns_to_dict(v) for k, v in vars(o).items()}}


def shape(o):
    """Attribute/key structure with leaf types (values dropped)."""
    if isinstance(o, dict):
        return {k: shape(v) for k, v in o.items() if k != "__type__"}
    if isinstance(o, list):
        return [shape(x) for x in o]
    return type(o).__name__


def contained(ref, got):
    """Every attribute of the reference structure exists in ours with the same leaf type (ours may
    carry extra attributes: score, row, file_id)."""
    if isinstance(ref, dict):
        return isinstance(got, dict) and all(k in got and contained(v, got[k]) for k, v in ref.items())
    if isinstance(ref, list):
        return isinstance(got, list) and len(ref) == len(got) and all(contained(a, b) for a, b in zip(ref, got))
    return ref == got


@pytest.fixture(scope="module")
def gold(golden_dir):
    return json.load(open(os.path.join(golden_dir, "ref_mock.json")))


def _contents(q):
    return [{"role": "user", "parts": [{"text": "earlier turn"}]}, {"role": "model", "parts": [{"text": "answer"}]},
            {"role": "user", "parts": [{"text": q}]}]


def test_fixture_is_the_reference_mock(gold):
    assert gold["client_type"] == "MockGeminiRag" and gold["is_mock"] is True
    assert gold["create_store"] == "fileSearchStores/mock-<hex32>"
    assert gold["upload_file"] == {"operation_name": "operations/mock-<hex32>", "file_id": "files/mock-<hex32>"}
    assert gold["op_status"] == {"name": "operations/mock-<hex32>", "done": True, "metadata": {}, "error": None}
    assert gold["op_status_dict_input"] == gold["op_status"]
    assert len(gold["cases"]) >= 12


def test_restatement_reproduces_reference(gold):
    for c in gold["cases"]:
        text = c["contents_to_text"]
        assert ns_to_dict(mock_ref.mock_response(text, c["store_names"])) == c["ask"]
        assert c["stream"][1] == c["ask"]  # the stream's second chunk is the same response
        assert c["stream"][0]["text"] == mock_ref.first_stream_text(text)
        assert c["stream"][0]["candidates"] is None
        assert mock_ref.extract_citations(mock_ref.mock_response(text, c["store_names"])) == c["citations"]


def test_adapter_contents_to_text_matches_reference(gold):
    for c in gold["cases"]:
        assert contents_to_text(_contents(c["question"])) == c["contents_to_text"]
    for s in gold["contents_to_text_shapes"]:
        assert contents_to_text(s["contents"]) == s["text"]


def test_local_adapter_boundary_matches_reference(gold, golden_dir):
    rag = LocalGpuRag(OracleRetriever(), top_k=1)
    st = rag.create_store("demo")
    rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md")
    for c in gold["cases"]:
        if not c["store_names"]:
            continue
        chunks = list(rag.ask_stream(contents=_contents(c["question"]), store_names=[st], metadata_filter=None,
                                     model="gemini-2.5-flash"))
        assert len(chunks) == len(c["stream"]) == 2
        assert ns_to_dict(chunks[0]) == c["stream"][0]  # first chunk: identical to the mock's
        ours = ns_to_dict(chunks[1])
        assert contained(shape(c["stream"][1]), shape(ours))
        cits = rag.extract_citations_from_response(chunks[1])
        ref = c["citations"]
        assert [sorted(x) for x in cits] == [sorted(x) for x in ref]
        assert [x["index"] for x in cits] == [0] and cits[0]["source_type"] == ref[0]["source_type"]
        assert cits[0]["store"] == st
    # no store: the mock invents "store/mock", the local backend has nothing to search
    chunks = list(rag.ask_stream(contents=_contents("q"), store_names=[], metadata_filter=None, model="m"))
    assert ns_to_dict(chunks[0]) == {"__type__": "SimpleNamespace", "text": "[mock-mode] q", "candidates": None,
                                     "usage_metadata": {"__type__": "SimpleNamespace", "prompt_token_count": 0,
                                                        "candidates_token_count": 0}}
    assert rag.extract_citations_from_response(chunks[1]) == []
    assert gold["cases"][1]["store_names"] == [] and gold["cases"][1]["citations"][0]["store"] == "store/mock"


def test_stream_ids_are_uuid4_pairs(gold):
    a, b = LocalGpuRag.new_stream_ids()
    assert gold["new_stream_ids_pattern"] == ["<hex32>", "<hex32>"]
    assert len(a.replace("-", "")) == 32 and len(b.replace("-", "")) == 32 and a != b
