"""Counter-based synthetic corpus/query generator (oracle restatement).

Bit-identical to rag-foundation_amd/csrc/k_scan_valu.hip:synth_rows_kernel:
  base = splitmix64(seed); u = splitmix64(base + row*dim + col)  (mod 2^64)
  n    = 2*(u >> 40) + 1 - 2^24              odd integer in (-2^24, 2^24)
  x    = f32( f64(n) * (1 / sqrt(f64(sum_row n^2))) )   then bf16/f16 by round-to-nearest-even
The row sum of squares is exact in int64 (n^2 < 2^48, dim <= 4096).
"""
import numpy as np

M64 = (1 << 64) - 1
_C1 = np.uint64(0x9E3779B97F4A7C15)
_C2 = np.uint64(0xBF58476D1CE4E5B9)
_C3 = np.uint64(0x94D049BB133111EB)


def splitmix64_int(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64) + _C1
    x = (x ^ (x >> np.uint64(30))) * _C2
    x = (x ^ (x >> np.uint64(27))) * _C3
    return x ^ (x >> np.uint64(31))


def raw_rows(seed: int, row0: int, n: int, dim: int) -> np.ndarray:
    """int64 [n][dim] odd integers n(seed,row,col)."""
    base = np.uint64(splitmix64_int(seed))
    idx = (np.arange(row0, row0 + n, dtype=np.uint64)[:, None] * np.uint64(dim)
           + np.arange(dim, dtype=np.uint64)[None, :])
    u = splitmix64(base + idx)
    return (2 * (u >> np.uint64(40)).astype(np.int64)) + 1 - (1 << 24)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even f32 -> bf16 bit pattern (uint16); NaN stays a quiet NaN."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def normalize_exact(nint: np.ndarray) -> np.ndarray:
    """f32 rows from int64 rows: f32(f64(n) * (1/sqrt(f64(sum n^2)))); zero rows stay zero."""
    ss = (nint * nint).sum(axis=1)
    r = np.zeros(ss.shape, dtype=np.float64)
    nz = ss > 0
    r[nz] = 1.0 / np.sqrt(ss[nz].astype(np.float64))
    return (nint.astype(np.float64) * r[:, None]).astype(np.float32)


def synth_rows(seed: int, row0: int, n: int, dim: int, dtype: str = "f32") -> np.ndarray:
    """Rows in the storage dtype: f32 array, bf16 as uint16 bits, f16 as float16."""
    x = normalize_exact(raw_rows(seed, row0, n, dim))
    if dtype == "f32":
        return x
    if dtype == "bf16":
        return f32_to_bf16_bits(x)
    if dtype == "f16":
        return x.astype(np.float16)
    raise ValueError(dtype)


def to_f64(rows: np.ndarray, dtype: str) -> np.ndarray:
    """Exact widening of stored rows to float64."""
    if dtype == "bf16":
        return bf16_bits_to_f32(rows).astype(np.float64)
    return np.asarray(rows).astype(np.float64)
