"""Text side of the index write (oracle restatement; see oracle/__init__.py for the rules).

normalize()          restates scripts/benchmark/metrics.py:13-19 (_normalize) — the only
                     tokeniser in the reference — and is pinned by tests/golden/ref_normalize.json
                     captured from the reference function itself.
contents_to_text()   restates MockGeminiRag._contents_to_text, gemini_rag.py:640-654.
chunk_whitespace()   Gemini white_space_config semantics (the reference forwards
                     chunking_config to Gemini, gemini_rag.py:324-326); build-defined.
featurize()          hashed bag of words (build-defined; C version: csrc/featurize.cpp).
"""
import re

import numpy as np

from .synth import splitmix64_int

ARTICLES = {"a", "an", "the"}
_WS = b" \t\n\x0b\x0c\r\x1c\x1d\x1e\x1f"
MAX_TOKENS_PER_CHUNK = 65536
M64 = (1 << 64) - 1


def normalize(text):
    """metrics.py:13-19: lower, [^a-z0-9\\s] -> ' ', split, drop articles, join with ' '."""
    if not text:
        return ""
    text = text.lower()
    text = re.sub(r"[^a-z0-9\s]", " ", text)
    tokens = [t for t in text.split() if t and t not in ARTICLES]
    return " ".join(tokens)


def tokens_bytes(b: bytes):
    """Byte-level restatement used by the index: after ASCII lower-casing, tokens are maximal
    runs of [a-z0-9]; articles dropped.  Equals normalize(text).split() for any text whose
    str.lower() has been applied first (non-ASCII bytes are >= 0x80, hence separators)."""
    low = bytes(c + 32 if 65 <= c <= 90 else c for c in b)
    toks = re.findall(rb"[a-z0-9]+", low)
    return [t for t in toks if t not in (b"a", b"an", b"the")]


def contents_to_text(contents):
    """gemini_rag.py:640-654."""
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


def chunk_whitespace(b: bytes, max_tokens: int, overlap: int):
    """[(start, end)] byte spans of windows of max_tokens whitespace tokens, overlap shared."""
    if not (1 <= max_tokens <= 65536 and 0 <= overlap < max_tokens):
        raise ValueError("bad chunking config")
    toks = [(m.start(), m.end()) for m in re.finditer(rb"[^" + re.escape(_WS) + rb"]+", b)]
    spans = []
    nt = len(toks)
    start = 0
    while nt > 0:
        end = min(start + max_tokens, nt)
        spans.append((toks[start][0], toks[end - 1][1]))
        if end == nt:
            break
        start = end - overlap
    return spans


def fnv1a64(t: bytes) -> int:
    h = 0xCBF29CE484222325
    for c in t:
        h ^= c
        h = (h * 0x100000001B3) & M64
    return h


def token_hash(t: bytes, hash_seed: int) -> int:
    return splitmix64_int((fnv1a64(t) + hash_seed) & M64)


def featurize(b: bytes, spans, V: int, hash_seed: int):
    """CSR (indptr int32, bucket int32, count int16): per chunk sorted unique buckets with signed
    counts (sign = top hash bit), zero counts dropped, clamped to [-256, 256]; at most 65536
    normalised tokens per chunk."""
    indptr = [0]
    buckets, counts = [], []
    for (s, e) in spans:
        toks = tokens_bytes(b[s:e])[:MAX_TOKENS_PER_CHUNK]
        acc = {}
        for t in toks:
            h = token_hash(t, hash_seed)
            bk = h & (V - 1)
            acc[bk] = acc.get(bk, 0) + (-1 if h >> 63 else 1)
        for bk in sorted(acc):
            c = acc[bk]
            if c == 0:
                continue
            buckets.append(bk)
            counts.append(max(-256, min(256, c)))
        indptr.append(len(buckets))
    return (np.array(indptr, dtype=np.int32), np.array(buckets, dtype=np.int32),
            np.array(counts, dtype=np.int16))
