"""ctypes binding of librfx.so (C ABI: include/rfx.h).

torch is imported first on purpose: torch bundles its own libamdhip64.so.7 and librfx.so links
the same SONAME, so the dynamic loader binds librfx to the runtime torch already loaded — one HIP
runtime per process, and device pointers / streams from torch are valid inside the library.

There is NO fallback: if librfx.so is missing or fails to load, importing this module raises.
"""
import ctypes
import hashlib
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RFX_LIB", os.path.join(_HERE, "librfx.so"))

RFX_OK, RFX_EINVAL, RFX_ENOMEM, RFX_EDEVICE, RFX_EIO, RFX_EBUSY, RFX_EUNSUPPORTED, RFX_ECAPACITY = range(8)
RFX_F32, RFX_BF16, RFX_F16 = 0, 1, 2

DTYPE_CODES = {"f32": RFX_F32, "bf16": RFX_BF16, "f16": RFX_F16}
TORCH_DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}
ESIZE = {"f32": 4, "bf16": 2, "f16": 2}


class RfxError(RuntimeError):
    """Non-transient library failure (maps to the reference's fatal-error handling:
    chat -> SSE unexpected_error frame chat.py:1130-1143; ingestion -> Document ERROR
    ingestion.py:311-339)."""

    def __init__(self, code, msg):
        super().__init__(f"rfx error {code}: {msg}")
        self.code = code


class RfxCapacityError(RfxError):
    """The int8 copy of the two-pass scan does not fit (RFX_ECAPACITY): the index stays exact.  Never
    an upload failure: rfx.store logs it and keeps answering with the exact scan."""


class RfxTransientError(TimeoutError):
    """Transient failure (device busy / queue timeout).  Subclasses TimeoutError so the
    reference's RETRYABLE_EXCEPTIONS (gemini_rag.py:22-27) retry it unchanged."""

    def __init__(self, code, msg):
        super().__init__(f"rfx transient error {code}: {msg}")
        self.code = code


if not os.path.exists(LIB_PATH):
    raise ImportError(f"librfx.so not found at {LIB_PATH}: build it with __graft_entry__.build() "
                      f"(make -C rag-foundation_amd/csrc); there is no CPU fallback")

lib = ctypes.CDLL(LIB_PATH)
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")


def source_hash() -> str:
    """sha256 (16 hex) of the library sources, computed exactly as csrc/Makefile does for the
    rfx_build_id() it bakes into librfx.so: *.hip *.h *.cpp in byte order, then the Makefile
    and include/rfx.h.  None when the sources are not shipped next to the library."""
    try:
        names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h", ".cpp")))
        paths = [os.path.join(CSRC, f) for f in names] + [os.path.join(CSRC, "Makefile"),
                                                           os.path.join(CSRC, "..", "..", "include", "rfx.h")]
        h = hashlib.sha256()
        for q in paths:
            with open(q, "rb") as f:
                h.update(f.read())
        return h.hexdigest()[:16]
    except OSError:
        return None


lib.rfx_build_id.argtypes = []
lib.rfx_build_id.restype = ctypes.c_char_p
BUILD_ID = lib.rfx_build_id().decode()
SOURCE_HASH = source_hash()
if SOURCE_HASH is not None and SOURCE_HASH != BUILD_ID and os.environ.get("RFX_ALLOW_STALE_LIB") != "1":
    raise ImportError(f"{LIB_PATH} was built from other sources (build id {BUILD_ID}, tree {SOURCE_HASH}): "
                      f"rebuild with __graft_entry__.build()")

_i = ctypes.c_int
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_p = ctypes.c_void_p
_sz = ctypes.c_size_t
_pi = ctypes.POINTER(ctypes.c_int)
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pu64 = ctypes.POINTER(ctypes.c_uint64)
_psz = ctypes.POINTER(ctypes.c_size_t)
_pp = ctypes.POINTER(ctypes.c_void_p)
_cs = ctypes.c_char_p

SIGNATURES = {
    "rfx_last_error": ([], ctypes.c_char_p),
    "rfx_version": ([], _i),
    "rfx_build_id": ([], ctypes.c_char_p),
    "rfx_device_count": ([_pi], _i),
    "rfx_init": ([_i], _i),
    "rfx_index_create": ([_i, _i, _i, _i64, _pu64], _i),
    "rfx_index_destroy": ([_u64], _i),
    "rfx_index_info": ([_u64, _pi, _pi, _pi64, _pi64, _pi64], _i),
    "rfx_union_create": ([_pu64, _i, _p, _pu64, _pi64], _i),
    "rfx_union_refresh": ([_u64, _p, _pi], _i),
    "rfx_index_reserve": ([_u64, _i64], _i),
    "rfx_index_add": ([_u64, _p, _i64, _i, _pi64, _p], _i),
    "rfx_index_add_synthetic": ([_u64, _u64, _i64, _i64, _pi64, _p], _i),
    "rfx_index_write": ([_u64, _i64, _p, _i64, _i, _p], _i),
    "rfx_index_tombstone": ([_u64, _pi64, _i64, _p], _i),
    "rfx_index_read": ([_u64, _i64, _i64, _p, _i, _p], _i),
    "rfx_index_data": ([_u64, _pp], _i),
    "rfx_index_save": ([_u64, _cs], _i),
    "rfx_index_load": ([_cs, _i, _pu64], _i),
    "rfx_rows_append": ([_u64, _cs, _i64, _i64], _i),
    "rfx_rows_sync": ([_u64, _cs, _i64, _i64], _i),
    "rfx_comm_unique_id": ([_p], _i),
    "rfx_comm_init_rank": ([_i, _i, _p, _i, _pu64], _i),
    "rfx_comm_init_all": ([_i, _p, _pu64], _i),
    "rfx_comm_info": ([_u64, _pi, _pi, _pi], _i),
    "rfx_comm_destroy": ([_u64], _i),
    "rfx_allgather_records": ([_u64, _p, _p, _i64, _i, _p], _i),
    "rfx_gather_records": ([_u64, _p, _p, _i, _i64, _i, _p], _i),
    "rfx_search_workspace_bytes": ([_u64, _i64, _i, _psz], _i),
    "rfx_search": ([_u64, _p, _i64, _i, _p, _p, _p, _sz, _p], _i),
    "rfx_scan_plan": ([_u64, _i64, _i, _pi, _pi64], _i),
    "rfx_scan_topk": ([_u64, _p, _i64, _i, _p, _p, _p, _sz, _p], _i),
    "rfx_synth_clustered": ([_u64, _i64, _u64, _i64, _i64, _i, _i, _p, _p], _i),
    "rfx_quantize": ([_p, _i64, _i, _i, _p, _p, _p], _i),
    "rfx_ivf_create": ([_i, _i, _i, _pu64], _i),
    "rfx_ivf_destroy": ([_u64], _i),
    "rfx_ivf_info": ([_u64, _pi, _pi, _pi64, _pi], _i),
    "rfx_ivf_train": ([_u64, _p, _i64, _i, _i, _p], _i),
    "rfx_ivf_set_centroids": ([_u64, _p, _p], _i),
    "rfx_ivf_get_centroids": ([_u64, _p, _p, _p], _i),
    "rfx_ivf_add": ([_u64, _p, _i64, _i, _p], _i),
    "rfx_ivf_build": ([_u64, _p], _i),
    "rfx_ivf_save": ([_u64, _cs], _i),
    "rfx_ivf_load": ([_cs, _i, _pu64], _i),
    "rfx_ivf_codes": ([_u64, _p, _p, _p, _p], _i),
    "rfx_ivf_lists": ([_u64, _p, _p, _p], _i),
    "rfx_ivf_search_workspace_bytes": ([_u64, _i64, _i, _i, _psz], _i),
    "rfx_ivf_rerank_workspace_bytes": ([_u64, _i64, _i, _i, _i, _psz], _i),
    "rfx_ivf_search_rerank": ([_u64, _p, _i64, _i, _i, _i, _i, _p, _i, _p, _p, _p, _sz, _p], _i),
    "rfx_rerank_candidates": ([_p, _i64, _i, _p, _i, _i64, _i64, _i, _p, _i, _p, _p, _p], _i),
    "rfx_ivf_search": ([_u64, _p, _i64, _i, _i, _i, _p, _p, _p, _sz, _p], _i),
    "rfx_search_masked": ([_u64, _p, _i64, _i, _p, _i64, _p, _p, _p, _sz, _p], _i),
    "rfx_search_records": ([_u64, _p, _i64, _i, _p, _i64, _i64, _p, _p, _sz, _p], _i),
    "rfx_search_plan": ([_u64, _i64, _i, _pi], _i),
    "rfx_rescore_topk": ([_u64, _p, _i64, _i, _i64, _p, _p, _p, _p], _i),
    "rfx_sharded_search": ([_i, _p, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _p], _i),
    "rfx_search_timed": ([_u64, _p, _i64, _i, _p, _i64, _i64, _p, _p, _p, _p, _sz, _p, _p, _p], _i),
    "rfx_search_staged": ([_u64, _p, _i64, _i, _p, _i64, _i64, _p, _p, _p, _p, _sz, _i, _i, _p], _i),
    "rfx_stream_create_cu_mask": ([_i, _p, _i, _pp], _i),
    "rfx_stream_destroy": ([_p], _i),
    "rfx_index_screen": ([_u64, _i, _p], _i),
    "rfx_index_screen_state": ([_u64, _pi, _pi64, _pi], _i),
    "rfx_index_screen_read": ([_u64, _i64, _i64, _p, _p, _p, _p], _i),
    "rfx_screen_diag": ([_u64, _i64, _i, _p, _p, _p], _i),
    "rfx_scan_topk_masked": ([_u64, _p, _i64, _i, _p, _i64, _p, _p, _p, _sz, _p], _i),
    "rfx_topk_merge": ([_p, _p, _i, _i64, _i64, _i, _i64, _p, _p, _p], _i),
    "rfx_scan_list_len": ([_u64, _i64, _i, _p], _i),
    "rfx_topk_merge_lists": ([_p, _p, _i, _i64, _i64, _i, _i, _i64, _p, _p, _p], _i),
    "rfx_topk_merge_records": ([_p, _p, _i, _i64, _i64, _i, _i, _i64, _p, _p], _i),
    "rfx_merge_gathered": ([_p, _i, _i64, _i, _p, _p, _p], _i),
    "rfx_topk_merge_sorted": ([_p, _p, _i, _i64, _i64, _i, _i, _i64, _p, _p, _p, _p], _i),
    "rfx_chunk_whitespace": ([_p, _i64, _i, _i, _p, _i64, _pi64], _i),
    "rfx_featurize": ([_p, _p, _i64, _i, _u64, _p, _p, _p, _i64, _pi64], _i),
    "rfx_embed_weights": ([_i, _i, _u64, _p, _p], _i),
    "rfx_embed_workspace_bytes": ([_i64, _i, _psz], _i),
    "rfx_embed": ([_p, _p, _p, _i64, _i, _p, _i, _p, _i, _p, _sz, _p], _i),
    "rfx_synth_rows": ([_u64, _i64, _i64, _i, _i, _p, _p], _i),
}

for _name, (_args, _res) in SIGNATURES.items():
    _f = getattr(lib, _name)  # AttributeError here = the library does not export a declared symbol
    _f.argtypes = _args
    _f.restype = _res


def check(rc: int, what: str = ""):
    """Raise on a non-zero status code."""
    if rc == RFX_OK:
        return
    msg = lib.rfx_last_error().decode(errors="replace") or what
    if rc == RFX_EBUSY:
        raise RfxTransientError(rc, msg)
    if rc == RFX_EINVAL:
        raise ValueError(f"rfx: {msg}")
    if rc == RFX_ECAPACITY:
        raise RfxCapacityError(rc, msg)
    raise RfxError(rc, msg)


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (default: the current stream of the current device)."""
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())
