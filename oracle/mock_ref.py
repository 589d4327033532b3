"""Restatement of the reference's mock retriever response shapes, used to check that the
local-GPU adapter's outputs have the reference structure.

  MockGeminiRag._mock_response        gemini_rag.py:704-718
  MockGeminiRag.ask_stream (2 chunks)  gemini_rag.py:673-694
  GeminiRag.extract_citations_...      gemini_rag.py:554-595
Pinned by tests/golden/ref_mock.json, captured from the reference in the build container.
"""
from types import SimpleNamespace


def mock_response(question, store_names):
    snippet = question[:128] if question else "Mock response"
    usage = SimpleNamespace(prompt_token_count=0, candidates_token_count=0)
    rc = SimpleNamespace(uri="mock://document", title="Mock Document", text=f"Mock snippet: {snippet}",
                         file_search_store=store_names[0] if store_names else "store/mock")
    cand = SimpleNamespace(grounding_metadata=SimpleNamespace(
        grounding_chunks=[SimpleNamespace(retrieved_context=rc, web=None)]), usage_metadata=usage)
    return SimpleNamespace(text=None, candidates=[cand], usage_metadata=usage)


def first_stream_text(text):
    return f"[mock-mode] {text or 'response'}"


def extract_citations(response):
    out = []
    try:
        cand = response.candidates[0]
        gm = getattr(cand, "grounding_metadata", None)
        if not gm:
            return out
        for i, ch in enumerate(list(getattr(gm, "grounding_chunks", []) or [])):
            rc = getattr(ch, "retrieved_context", None)
            if rc:
                out.append({"index": i, "source_type": "retrieved_context", "uri": getattr(rc, "uri", None),
                            "title": getattr(rc, "title", None), "snippet": getattr(rc, "text", None),
                            "store": getattr(rc, "file_search_store", None)})
                continue
            web = getattr(ch, "web", None)
            if web:
                out.append({"index": i, "source_type": "web", "uri": getattr(web, "uri", None),
                            "title": getattr(web, "title", None), "snippet": None, "store": None})
        return out
    except (AttributeError, KeyError, IndexError, TypeError):
        return out
