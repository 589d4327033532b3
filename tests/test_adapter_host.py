"""CPU: the adapter's host logic against the reference boundary, with an oracle-backed
retriever injected (tests/fakes.py).  The product default is GpuRetriever (HIP only)."""
import json
import os
import uuid

import pytest

from fakes import OracleRetriever
from oracle import mock_ref
from rfx.adapter import LocalGpuRag, UploadResult, build_response, contents_to_text, get_rag_client


@pytest.fixture()
def rag():
    return LocalGpuRag(OracleRetriever(), top_k=5)


@pytest.fixture()
def store_with_doc(rag, golden_dir):
    st = rag.create_store("demo")
    up = rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md",
                         chunking_config={"white_space_config": {"max_tokens_per_chunk": 3, "max_overlap_tokens": 0}})
    return st, up


def test_is_mock_truthy_for_health(rag):
    assert rag.is_mock  # main.py:385 skips the external probe


def test_create_store_name_prefix(rag):
    name = rag.create_store("x")
    assert name.startswith("fileSearchStores/") and len(name) <= 255  # stores.py:46, models.py:66


def test_upload_file_contract(rag, store_with_doc):
    st, up = store_with_doc
    assert isinstance(up, UploadResult)
    assert up.operation_name.startswith("operations/") and len(up.operation_name) <= 255
    assert up.file_id.startswith("files/") and len(up.file_id) <= 255
    # ingestion.py:52 calls upload_file(fs_name, path, display_name=...) positionally
    up2 = rag.upload_file(st, os.path.join(os.path.dirname(__file__), "golden", "sample_report.md"), display_name=None)
    assert up2.file_id != up.file_id


def test_op_status_shape(rag):
    st = rag.op_status("operations/local-abc")
    assert st == {"name": "operations/local-abc", "done": True, "metadata": {}, "error": None}
    assert rag.op_status({"name": "operations/x"})["name"] == "operations/x"
    with pytest.raises(ValueError):
        rag.op_status({})


def test_ask_stream_two_chunks_and_first_text_parity(rag, store_with_doc):
    st, _ = store_with_doc
    q = "How are uploaded documents ingested?"
    contents = [{"role": "user", "parts": [{"text": "earlier turn"}]}, {"role": "user", "parts": [{"text": q}]}]
    chunks = list(rag.ask_stream(contents=contents, store_names=[st], metadata_filter=None, model="gemini-2.5-flash"))
    assert len(chunks) == 2
    assert chunks[0].text == mock_ref.first_stream_text(q) and chunks[0].candidates is None
    assert chunks[0].usage_metadata.prompt_token_count == 0
    assert chunks[1].candidates  # chat.py:1056 treats the chunk with candidates as final_resp


def test_citations_rank_order_and_keys(rag, store_with_doc, golden_dir):
    st, _ = store_with_doc
    fx = json.load(open(os.path.join(golden_dir, "cfg1_sample_report.json")))
    for case in fx["queries"]:
        resp = rag.ask(contents=case["question"], store_names=[st], metadata_filter=None, model="m")
        cits = rag.extract_citations_from_response(resp)
        ref_keys = set(mock_ref.extract_citations(mock_ref.mock_response("q", [st]))[0])
        assert all(set(c) == ref_keys for c in cits)
        assert [c["index"] for c in cits] == list(range(len(cits)))
        assert [c["snippet"] for c in cits] == case["snippets"]
        assert all(c["store"] == st and c["source_type"] == "retrieved_context" for c in cits)
        gc = resp.candidates[0].grounding_metadata.grounding_chunks
        assert [g.retrieved_context.row for g in gc] == case["rows"]


def test_citation_frames_wire_format(rag, store_with_doc):
    """Same mapping as chat.py:_citation_frames (576-586)."""
    st, _ = store_with_doc
    resp = rag.ask(contents="demo flow", store_names=[st], metadata_filter=None, model="m")
    for c in rag.extract_citations_from_response(resp):
        payload = {"type": "source-document", "sourceId": f"cit-{c['index']}", "mediaType": "file",
                   "title": c.get("title") or c.get("uri") or "Source", "snippet": c.get("snippet")}
        assert payload["title"] == "sample-report.md" and payload["snippet"]


def test_metadata_filter_ignored_when_disabled(rag, store_with_doc):
    # RFX_METADATA_FILTER=0: the reference mock's behaviour (filter accepted and ignored)
    st, _ = store_with_doc
    rag.apply_filters = False
    a = rag.ask(contents="demo", store_names=[st], metadata_filter={"tenant": "acme", "region": ["a", "b"]}, model="m")
    b = rag.ask(contents="demo", store_names=[st], metadata_filter=None, model="m")
    assert rag.extract_citations_from_response(a) == rag.extract_citations_from_response(b)


def _two_tenant_store(rag, tmp_path):
    st = rag.create_store("tenants")
    ids = {}
    for tenant, words in (("acme", "alpha beta gamma delta " * 8), ("globex", "alpha beta epsilon zeta " * 8)):
        p = tmp_path / f"{tenant}.txt"
        p.write_text(words)
        up = rag.upload_file(st, str(p), display_name=f"{tenant}.txt",
                             custom_metadata=[{"key": "tenant", "string_value": tenant},
                                              {"key": "year", "numeric_value": 2024 if tenant == "acme" else 2025}],
                             chunking_config={"white_space_config": {"max_tokens_per_chunk": 4, "max_overlap_tokens": 0}})
        ids[tenant] = up.file_id
    return st, ids


def test_metadata_filter_selects_files(rag, tmp_path):
    st, ids = _two_tenant_store(rag, tmp_path)

    def titles(filt, k=20):
        r = rag.ask(contents="alpha beta", store_names=[st], metadata_filter=filt, model="m", top_k=k)
        return [c["title"] for c in rag.extract_citations_from_response(r)]

    everything = titles(None)
    assert set(everything) == {"acme.txt", "globex.txt"}
    assert titles({"tenant": "acme"}) == [t for t in everything if t == "acme.txt"]
    assert titles({"tenant": ["acme", "globex"]}) == everything
    assert titles({"year": 2025}) == [t for t in everything if t == "globex.txt"]
    assert titles({"year": 2025.0, "tenant": "globex"}) == [t for t in everything if t == "globex.txt"]
    assert titles({"tenant": "acme", "year": 2025}) == []  # AND over keys
    assert titles({"tenant": "initech"}) == []
    assert titles({"missing_key": "x"}) == []
    with pytest.raises(ValueError):
        titles("tenant=acme")
    with pytest.raises(ValueError):
        titles({"tenant": []})


def test_top_k_end_to_end(rag, tmp_path):
    st, _ = _two_tenant_store(rag, tmp_path)
    q = [{"role": "user", "parts": [{"text": "alpha beta"}]}]
    for k in (1, 3, 7, 16):
        chunks = list(rag.ask_stream(contents=q, store_names=[st], metadata_filter=None, model="m", top_k=k))
        assert len(chunks[1].candidates[0].grounding_metadata.grounding_chunks) == k
    default = list(rag.ask_stream(contents=q, store_names=[st], metadata_filter=None, model="m"))
    assert len(default[1].candidates[0].grounding_metadata.grounding_chunks) == rag.top_k
    for bad in (0, 65):
        with pytest.raises(ValueError):
            list(rag.ask_stream(contents=q, store_names=[st], metadata_filter=None, model="m", top_k=bad))


def test_empty_and_unknown_stores(rag):
    resp = rag.ask(contents="anything", store_names=[], metadata_filter=None, model="m")
    assert rag.extract_citations_from_response(resp) == []
    resp = rag.ask(contents="anything", store_names=["fileSearchStores/local-missing"], metadata_filter=None, model="m")
    assert rag.extract_citations_from_response(resp) == []


def test_multi_store_union_is_rank_ordered(rag, golden_dir):
    a, b = rag.create_store("a"), rag.create_store("b")
    path = os.path.join(golden_dir, "sample_report.md")
    cfg = {"white_space_config": {"max_tokens_per_chunk": 5, "max_overlap_tokens": 1}}
    rag.upload_file(a, path, display_name="A", chunking_config=cfg)
    rag.upload_file(b, path, display_name="B", chunking_config=cfg)
    hits = rag.retrieve("chat answers stream back with citations", [a, b], k=6)
    scores = [h.score for h in hits]
    assert scores == sorted(scores, reverse=True)
    # identical documents: each tie pair comes back store a first
    for i in range(0, 6, 2):
        assert hits[i].store == a and hits[i + 1].store == b and hits[i].row == hits[i + 1].row


def test_delete_document_semantics(rag, store_with_doc):
    st, up = store_with_doc
    rag.delete_document_from_store(st, 1, "sample-report.md", file_id=None)  # no file id -> skip
    assert rag.retrieve("uploaded documents", [st])
    rag.delete_document_from_store(st, 1, "sample-report.md", file_id=up.file_id)
    assert rag.retrieve("uploaded documents", [st]) == []
    rag.delete_document_from_store(st, 1, "sample-report.md", file_id=up.file_id)  # already gone = success
    rag.delete_document_from_store("fileSearchStores/local-nope", 1, file_id="files/x")  # 404 = success


def test_delete_store(rag, store_with_doc):
    st, _ = store_with_doc
    rag.delete_store(st)
    assert st not in [s.name for s in rag.list_stores()]
    rag.delete_store("")  # no-op like the reference


def test_new_stream_ids():
    a, b = LocalGpuRag.new_stream_ids()
    assert a != b and len(a) == 36 and len(b) == 36 and uuid.UUID(a)


def test_extract_citations_robustness(caplog):
    from unittest.mock import Mock
    assert LocalGpuRag.extract_citations_from_response(Mock(candidates=[])) == []
    assert LocalGpuRag.extract_citations_from_response(Mock(candidates=[Mock(grounding_metadata=None)])) == []
    with caplog.at_level("WARNING"):
        assert LocalGpuRag.extract_citations_from_response(Mock(spec=[])) == []
    assert "Failed to extract citations" in caplog.text
    web = Mock(retrieved_context=None, web=Mock(uri="u", title="t"))
    out = LocalGpuRag.extract_citations_from_response(Mock(candidates=[Mock(grounding_metadata=Mock(grounding_chunks=[web]))]))
    assert out == [{"index": 0, "source_type": "web", "uri": "u", "title": "t", "snippet": None, "store": None}]


def test_extract_citations_same_as_reference_restatement():
    resp = mock_ref.mock_response("hello", ["fileSearchStores/s"])
    assert LocalGpuRag.extract_citations_from_response(resp) == mock_ref.extract_citations(resp)


def test_contents_to_text_matches_oracle():
    from oracle import textproc
    for c in ["x", [{"parts": [{"text": "a"}]}], [], [{"parts": "bad"}, "  s  "], 12]:
        assert contents_to_text(c) == textproc.contents_to_text(c)


def test_build_response_empty():
    resp = build_response([], [])
    assert LocalGpuRag.extract_citations_from_response(resp) == []


def test_errors_map_to_reference_retry_classes():
    from rfx._lib import RfxError, RfxTransientError
    assert issubclass(RfxTransientError, TimeoutError)  # in RETRYABLE_EXCEPTIONS (gemini_rag.py:22-27)
    assert not issubclass(RfxError, TimeoutError)


def test_get_rag_client_is_hip_backed():
    """The product factory builds the GPU retriever (no CPU fallback to the oracle)."""
    rag = get_rag_client()
    from rfx.retriever import GpuRetriever
    assert isinstance(rag.retriever, GpuRetriever)
