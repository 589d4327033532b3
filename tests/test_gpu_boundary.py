"""GPU: LocalGpuRag (HIP path) on the config-1 store, k = 1 and k = 5, against the reference's own
boundary vectors (tests/golden/ref_boundary.json): the citations it yields become chat-route
payloads (oracle.mock_ref restatement of chat.py:576-603, pinned by the reference's test) with
exactly the reference payload's shape, in rank order, carrying the oracle's top-k rows
(tests/golden/cfg1_sample_report.json)."""
import json
import os

import pytest

from oracle import mock_ref
from test_boundary_golden import payload_shape_ok

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_cfg1_frames_k1_k5(golden_dir, tmp_path, dtype):
    from rfx import store as rstore
    from rfx.adapter import LocalGpuRag
    from rfx.retriever import GpuRetriever

    gold = json.load(open(os.path.join(golden_dir, "ref_boundary.json")))
    fx = json.load(open(os.path.join(golden_dir, "cfg1_sample_report.json")))
    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path), device=0))
    rag = LocalGpuRag(GpuRetriever(dtype=dtype))
    st = rag.create_store("demo")
    rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md",
                    chunking_config={"white_space_config": fx["chunking"]})
    for case in fx["queries"]:
        for k in (1, 5):
            chunks = list(rag.ask_stream(contents=[{"role": "user", "parts": [{"text": case["question"]}]}],
                                         store_names=[st], metadata_filter=None, model="gemini-2.5-flash", top_k=k))
            assert chunks[0].text == mock_ref.first_stream_text(case["question"])
            cits = rag.extract_citations_from_response(chunks[1])
            gc = chunks[1].candidates[0].grounding_metadata.grounding_chunks
            if dtype == "f32":  # the fixture's oracle rows are for the f32 store
                assert [g.retrieved_context.row for g in gc] == case["rows"][:k]
            assert [c["snippet"] for c in cits] == [g.retrieved_context.text for g in gc]
            payload_shape_ok(mock_ref.citation_frame_payloads(cits), gold["citation_frame"]["payload"],
                             ["sample-report.md"] * k, [g.retrieved_context.text for g in gc])
            assert all(c["store"] == st for c in cits)
    rag.delete_store(st)


def test_multi_store_union_on_gpu(golden_dir, tmp_path):
    """ask_stream over several stores (gemini_rag.py:463-469 store_names list): the hits are the
    union's top-k in (score desc, store order, row asc); every hit's score is within 1e-5 of the
    oracle's f64 score of that chunk (oracle embedder, bit-exact with the GPU one)."""
    import numpy as np

    from fakes import OracleRetriever
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path), device=0))
    ret = GpuRetriever(dtype="f32")
    orc = OracleRetriever()
    text = open(os.path.join(golden_dir, "sample_report.md"), encoding="utf-8").read()
    docs = [text, "mock mode document assistant citations retrieval " * 12, text.upper(), "unrelated words " * 30]
    names = [ret.create_store(f"s{i}") for i in range(3)]
    for i, d in enumerate(docs):
        ret.add_document(names[i % 3], d, f"d{i}", {"white_space_config": {"max_tokens_per_chunk": 4,
                                                                            "max_overlap_tokens": 1}})
    for q in ["document assistant citations", "sample report", "unrelated"]:
        for k in (1, 5, 12):
            hits = ret.search(names, q, k)
            singles = [(h.score, si, h.row) for si, n in enumerate(names) for h in ret.search([n], q, k)]
            want = sorted(singles, key=lambda t: (-t[0], t[1], t[2]))[:k]
            assert [(h.score, names.index(h.store), h.row) for h in hits] == want
            qv = orc._embed([q])[0]
            for h in hits:
                ref = float(orc._embed([h.text])[0] @ qv)
                assert abs(h.score - ref) <= 1e-5, (h.text, h.score, ref)
            assert np.all(np.diff([h.score for h in hits]) <= 0)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_reference_mock_fixture_on_gpu(golden_dir, tmp_path, dtype):
    """The reference mock's captured outputs (tests/golden/ref_mock.json, MockGeminiRag) against
    LocalGpuRag on the HIP path at k = 1: the first stream chunk is identical; the second carries the
    mock's attribute structure, citation keys, rank-0 index and the queried store."""
    from rfx import store as rstore
    from rfx.adapter import LocalGpuRag
    from rfx.retriever import GpuRetriever
    from test_ref_mock_golden import _contents, contained, ns_to_dict, shape

    gold = json.load(open(os.path.join(golden_dir, "ref_mock.json")))
    rstore.set_registry(rstore.StoreRegistry(root=str(tmp_path), device=0))
    rag = LocalGpuRag(GpuRetriever(dtype=dtype), top_k=1)
    st = rag.create_store("demo")
    rag.upload_file(st, os.path.join(golden_dir, "sample_report.md"), display_name="sample-report.md")
    for c in gold["cases"]:
        if not c["store_names"]:
            continue
        chunks = list(rag.ask_stream(contents=_contents(c["question"]), store_names=[st], metadata_filter=None,
                                     model="gemini-2.5-flash"))
        assert ns_to_dict(chunks[0]) == c["stream"][0]
        assert contained(shape(c["stream"][1]), shape(ns_to_dict(chunks[1])))
        cits = rag.extract_citations_from_response(chunks[1])
        assert [sorted(x) for x in cits] == [sorted(x) for x in c["citations"]]
        assert cits[0]["index"] == 0 and cits[0]["store"] == st
    rag.delete_store(st)
