"""LocalGpuRag — drop-in Retriever/LLM adapter backed by the MI355X retrieval path.

Mirrors the duck-typed surface of the reference adapter
(backend/app/services/gemini_rag.py: GeminiRag 242-599, MockGeminiRag 602-718, get_rag_client
721-725) as its callers use it:
  create_store(display_name) -> "fileSearchStores/…"              stores.py:39
  upload_file(store, path, *, display_name, custom_metadata, chunking_config) -> UploadResult
                                                                  ingestion.py:52
  op_status(op) -> {name, done, metadata, error}                  ingestion.py:119, uploads.py:335
  ask_stream(*, contents, store_names, metadata_filter, model, system, top_k=None) -> 2 chunks
                                                                  chat.py:499-505
    (metadata_filter -> row mask, rfx.filters; top_k: the request's k, §8f item 3)
  ask(...) -> response                                            (interface completeness)
  extract_citations_from_response(resp) -> [citation dicts]       chat.py:578
  new_stream_ids() -> (uuid4, uuid4)                              chat.py:979
  delete_store(name) / delete_document_from_store(store, doc_id, filename=None, file_id=None)
                                                                  cleanup.py:37,66,122
  list_stores(); is_mock (truthy: /health skips the Gemini probe, main.py:385)
Streams keep the mock's exact first chunk ("[mock-mode] …", gemini_rag.py:686-690); the second
chunk carries the top-k retrieved chunks, in rank order, as grounding chunks (the reference
mock returns a single canned one, gemini_rag.py:704-718).  The LLM generation step is out of
scope (no model runs in the reference either).
"""
import logging
import os
import time
import uuid
from dataclasses import dataclass
from types import SimpleNamespace
from typing import Any, List, Optional, Sequence

from .metrics import observe

logger = logging.getLogger(__name__)


@dataclass
class UploadResult:
    """gemini_rag.py:30-33."""

    operation_name: str
    file_id: Optional[str] = None


def _get_response_name(response: Any, *, context: str) -> str:
    """gemini_rag.py:96-102."""
    if isinstance(response, str):
        return response
    name = response.get("name") if isinstance(response, dict) else getattr(response, "name", None)
    if not name:
        raise ValueError(f"Missing name in {context} response")
    return name


def contents_to_text(contents: Any) -> str:
    """Query text = last non-empty user text (MockGeminiRag._contents_to_text,
    gemini_rag.py:640-654)."""
    if isinstance(contents, str):
        return contents
    if isinstance(contents, list):
        for item in reversed(contents):
            if isinstance(item, str) and item.strip():
                return item.strip()
            if isinstance(item, dict):
                parts = item.get("parts")
                if isinstance(parts, list) and parts and isinstance(parts[0], dict):
                    text = parts[0].get("text")
                    if isinstance(text, str) and text.strip():
                        return text.strip()
    return str(contents)


def build_response(hits, store_names: Sequence[str]):
    """Response object with one grounding chunk per hit, in rank order.  Same attribute shape as
    MockGeminiRag._mock_response (gemini_rag.py:704-718); `score`, `row` and `file_id` are extra
    attributes the reference shape lacks (callers ignore unknown attributes)."""
    usage = SimpleNamespace(prompt_token_count=0, candidates_token_count=0)
    chunks = []
    for h in hits:
        rc = SimpleNamespace(uri=f"{h.uri}#chunk-{h.row}", title=h.title, text=h.text, file_search_store=h.store,
                             score=h.score, row=h.row, file_id=h.file_id)
        chunks.append(SimpleNamespace(retrieved_context=rc, web=None))
    cand = SimpleNamespace(grounding_metadata=SimpleNamespace(grounding_chunks=chunks), usage_metadata=usage)
    return SimpleNamespace(text=None, candidates=[cand], usage_metadata=usage)


class LocalGpuRag:
    """Thread-safe: all GPU state lives in the process-wide StoreRegistry."""

    def __init__(self, retriever=None, top_k: Optional[int] = None) -> None:
        if retriever is None:
            from .retriever import GpuRetriever  # imports the HIP library (fails loudly if absent)
            retriever = GpuRetriever()
        self.retriever = retriever
        self.top_k = int(os.environ.get("RFX_TOP_K", "5")) if top_k is None else int(top_k)
        # metadata filters become row masks; RFX_METADATA_FILTER=0 ignores them
        # like the reference mock (gemini_rag.py:673-694)
        self.apply_filters = os.environ.get("RFX_METADATA_FILTER", "1") != "0"
        self.is_mock = True

    # -------- Stores --------
    def list_stores(self) -> List[Any]:
        return [SimpleNamespace(name=n) for n in self.retriever.store_names()]

    def create_store(self, display_name: str) -> str:
        with observe("create_store"):
            return self.retriever.create_store(display_name)

    # -------- Upload & Operations --------
    def upload_file(self, store_name: str, file_path: str, *, display_name: Optional[str] = None,
                    custom_metadata=None, chunking_config=None) -> UploadResult:
        with observe("upload"):
            with open(file_path, "rb") as f:
                text = f.read().decode("utf-8", errors="replace")
            file_id, _ = self.retriever.add_document(store_name, text, display_name or os.path.basename(file_path),
                                                     chunking_config, custom_metadata)
            return UploadResult(operation_name=f"operations/local-{uuid.uuid4().hex}", file_id=file_id)

    def op_status(self, op_name) -> dict:
        """The index write is synchronous, so every operation is already done (the mock's answer,
        gemini_rag.py:631-638)."""
        name = _get_response_name(op_name, context="local operation status request")
        return {"name": name, "done": True, "metadata": {}, "error": None}

    def delete_store(self, store_name: str) -> None:
        if not store_name:
            return
        self.retriever.drop_store(store_name)

    def delete_document_from_store(self, store_name: str, document_id: int, filename: Optional[str] = None,
                                   file_id: Optional[str] = None) -> None:
        """Tombstones the file's rows; no file_id -> skip; unknown -> success (404 semantics,
        gemini_rag.py:392-424)."""
        if not file_id:
            logger.info("No file id recorded; skipping local delete", extra={"store": store_name,
                                                                               "document_id": document_id})
            return
        self.retriever.delete_file(store_name, file_id)

    # -------- Query (sync & stream) --------
    def retrieve(self, question: str, store_names: Sequence[str], k: Optional[int] = None,
                 metadata_filter: Optional[Any] = None):
        """Top-k hits.  k: the request's top_k (the reference route drops it,
        chat.py:66), default self.top_k; 1..64."""
        filt = metadata_filter if self.apply_filters else None
        return self.retriever.search(list(store_names or []), question, self.top_k if k is None else int(k),
                                     metadata_filter=filt)

    def ask(self, *, contents: Any, store_names: Sequence[str], metadata_filter: Optional[Any], model: str,
            system: Optional[str] = None, top_k: Optional[int] = None) -> Any:
        with observe("generate"):
            hits = self.retrieve(contents_to_text(contents), store_names, top_k, metadata_filter)
            return build_response(hits, store_names)

    def ask_stream(self, *, contents: Any, store_names: Sequence[str], metadata_filter: Optional[Any], model: str,
                   system: Optional[str] = None, top_k: Optional[int] = None):
        """The reference's keyword set plus an optional top_k (callers that do not pass it get
        self.top_k, so the reference call site chat.py:499-505 works unchanged)."""
        with observe("generate_stream"):
            text = contents_to_text(contents)
            resp = build_response(self.retrieve(text, store_names, top_k, metadata_filter), store_names)
        yield SimpleNamespace(text=f"[mock-mode] {text or 'response'}", candidates=None,
                              usage_metadata=SimpleNamespace(prompt_token_count=0, candidates_token_count=0))
        yield resp

    # -------- Citations --------
    @staticmethod
    def extract_citations_from_response(response: Any) -> List[dict]:
        """Same mapping as GeminiRag.extract_citations_from_response (gemini_rag.py:554-595)."""
        out: List[dict] = []
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
        except (AttributeError, KeyError, IndexError, TypeError) as e:
            logging.warning(f"Failed to extract citations: {e}",
                            extra={"response_type": type(response).__name__,
                                   "has_candidates": hasattr(response, "candidates")})
            return out

    @staticmethod
    def new_stream_ids() -> tuple:
        return str(uuid.uuid4()), str(uuid.uuid4())


def get_rag_client() -> LocalGpuRag:
    """Factory with the reference's signature (gemini_rag.py:721-725); a new lightweight
    instance per call, sharing the process-wide GPU state."""
    return LocalGpuRag()
