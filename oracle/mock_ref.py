"""Restatement of the reference's mock retriever response shapes, used to check that the
local-GPU adapter's outputs have the reference structure.

  MockGeminiRag._mock_response        gemini_rag.py:704-718
  MockGeminiRag.ask_stream (2 chunks)  gemini_rag.py:673-694
  GeminiRag.extract_citations_...      gemini_rag.py:554-595
  chat._citation_frames / _finish_frame chat.py:576-603 (the SSE payloads the chat route builds
                                        from the adapter's citations and usage)
Pinning: extract_citations, citation_frame_payloads and finish_frame_payload are checked against
the reference's own test vectors (tests/golden/ref_boundary.json, extracted from
backend/tests/test_gemini_rag.py and backend/tests/test_chat_stream_helpers.py by
tests/golden/make_ref_boundary.py).  mock_response / first_stream_text are pinned by the reference
MockGeminiRag's own outputs for a fixed question list (tests/golden/ref_mock.json, captured by
tests/golden/make_ref_mock.py; tests/test_ref_mock_golden.py).
"""
import json
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


def citation_frame_payloads(citations):
    """chat._citation_frames (chat.py:576-586): one "source-document" payload per citation."""
    return [{"type": "source-document", "sourceId": f"cit-{c['index']}", "mediaType": "file",
             "title": c.get("title") or c.get("uri") or "Source", "snippet": c.get("snippet")} for c in citations]


def citation_frames(citations):
    """The SSE frames themselves ("data: <json>\n\n")."""
    return [f"data: {json.dumps(p)}\n\n" for p in citation_frame_payloads(citations)]


def finish_frame_payload(*, prompt_tokens, completion_tokens, model):
    """chat._finish_frame (chat.py:589-603)."""
    return {"type": "finish", "finishReason": "stop", "promptTokens": prompt_tokens,
            "completionTokens": completion_tokens,
            "usage": {"prompt_tokens": prompt_tokens, "completion_tokens": completion_tokens, "model": model}}


def harness_citations(frames):
    """The benchmark harness's reading of a chat stream (scripts/benchmark/run_benchmark.py:
    196-216): every "source-document" frame becomes {title, snippet, sourceId}."""
    out = []
    for f in frames:
        if not f.startswith("data:") or f.strip() == "data: [DONE]":
            continue
        p = json.loads(f.split(": ", 1)[1])
        if p.get("type") == "source-document":
            out.append({"title": p.get("title"), "snippet": p.get("snippet"), "sourceId": p.get("sourceId")})
    return out
