"""Metadata filters -> row masks.

The reference accepts a metadata filter on chat requests and forwards it untouched to the
retrieval tool: `_validate_metadata_filter` (backend/app/routes/chat.py:295-335) allows
`{key: scalar | [scalar, ...]}` for allow-listed keys (scalars: str, int, float, bool;
`_coerce_metadata_value` :266-292), and `ask_stream(metadata_filter=...)` passes it to Gemini's
FileSearch tool (gemini_rag.py:463-469).  Documents carry metadata from upload
(`custom_metadata`, gemini_rag.py:314,324: a list of `{"key", "string_value" | "numeric_value"}`).
The mock ignores the filter (gemini_rag.py:673-694).

Here a filter selects files, and the selected files' row ranges become a device bitmap that the
scan kernels apply per tile (rfx_search_masked).  Semantics (Gemini's own matching is not
observable offline: parity unpinned against it):
  - a file matches when EVERY key of the filter matches (AND over keys);
  - a key matches when the file has that key and its value equals the filter scalar, or equals
    one of the filter list's values (OR within a list);
  - strings compare exactly; numbers (int/float) compare numerically; bools match only bools.
"""
import json
from typing import Any, Dict, Iterable, Optional, Tuple

import numpy as np

_SCALARS = (str, int, float, bool)


def normalize_metadata(custom_metadata: Any) -> Dict[str, Any]:
    """Upload metadata -> {key: value}.  Accepts Gemini's list form
    ([{"key": k, "string_value": v} | {"key": k, "numeric_value": n}], gemini_rag.py:314) or a
    plain dict.  Entries without a key or a scalar value are dropped."""
    out: Dict[str, Any] = {}
    if not custom_metadata:
        return out
    if isinstance(custom_metadata, dict):
        items = custom_metadata.items()
    else:
        items = []
        for e in custom_metadata:
            if not isinstance(e, dict) or not isinstance(e.get("key"), str):
                continue
            for vk in ("string_value", "numeric_value", "value"):
                if vk in e:
                    items.append((e["key"], e[vk]))
                    break
    for k, v in items:
        if isinstance(k, str) and k.strip() and isinstance(v, _SCALARS):
            out[k.strip()] = v
    return out


def _eq(a: Any, b: Any) -> bool:
    if isinstance(a, bool) or isinstance(b, bool):
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return float(a) == float(b)
    return isinstance(a, str) and isinstance(b, str) and a == b


def file_matches(metadata: Dict[str, Any], metadata_filter: Dict[str, Any]) -> bool:
    for key, want in metadata_filter.items():
        if key not in metadata:
            return False
        have = metadata[key]
        if isinstance(want, (list, tuple)):
            if not any(_eq(have, w) for w in want):
                return False
        elif not _eq(have, want):
            return False
    return True


def check_filter(metadata_filter: Any) -> Optional[Dict[str, Any]]:
    """None / {} -> None (no filter).  Otherwise the dict shape chat.py:295-335 lets through;
    anything else raises ValueError (the route answers 400 before the adapter is reached)."""
    if metadata_filter is None or metadata_filter == {}:
        return None
    if not isinstance(metadata_filter, dict):
        raise ValueError("metadata_filter must be a dict {key: scalar | [scalar, ...]}")
    for k, v in metadata_filter.items():
        if not isinstance(k, str) or not k.strip():
            raise ValueError("metadata_filter keys must be non-empty strings")
        vals = v if isinstance(v, list) else [v]
        if not vals or not all(isinstance(x, _SCALARS) for x in vals):
            raise ValueError(f"metadata_filter value for {k!r} must be a scalar or a non-empty list of scalars")
    return {k.strip(): v for k, v in metadata_filter.items()}


def filter_key(metadata_filter: Optional[Dict[str, Any]]) -> str:
    """Canonical string of a filter (cache and batching key); '' = no filter."""
    if metadata_filter is None:
        return ""
    return json.dumps(metadata_filter, sort_keys=True, separators=(",", ":"))


def row_mask_words(n_rows: int, ranges: Iterable[Tuple[int, int]]) -> np.ndarray:
    """Bitmap of (first, count) row ranges: int32 words, bit (r & 31) of word r >> 5 = row r
    (the layout rfx_search_masked reads), (n_rows + 31) // 32 words (at least one)."""
    allowed = np.zeros(max(1, (n_rows + 31) // 32) * 32, dtype=np.uint8)
    for first, count in ranges:
        if count > 0:
            allowed[first:first + count] = 1
    return np.packbits(allowed, bitorder="little").view("<u4").astype(np.uint32).view(np.int32)
