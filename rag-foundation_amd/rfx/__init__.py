"""rfx — MI355X-native embedding index + top-k retrieval behind the rag-foundation adapter API.

Importing the package is cheap; the HIP library is loaded by rfx._lib (imported by index,
embedder, retriever).  The adapter module itself only needs the library when a LocalGpuRag is
constructed without an injected retriever.
"""
from .adapter import LocalGpuRag, UploadResult, build_response, contents_to_text, get_rag_client  # noqa: F401

__all__ = ["LocalGpuRag", "UploadResult", "get_rag_client", "build_response", "contents_to_text"]
