"""Chunk embedding (oracle restatement of csrc/k_embed.hip), exact integer arithmetic.

W^T[j][v] = w/128 with w = ((u >> 32) * 255 >> 32) - 127, u = splitmix64(splitmix64(seed) + j*V + v)
e = F_int @ W_int  (int64, exact; equals 128 * the GPU's f32 MFMA result, which is exact)
x = f32( f64(e) * (1/sqrt(f64(sum e^2))) ), zero rows stay zero; then the index dtype.
"""
import numpy as np

from .synth import splitmix64, splitmix64_int, normalize_exact, f32_to_bf16_bits


def weights_int(V: int, dim: int, seed: int) -> np.ndarray:
    """int64 [dim][V] in [-127, 127] (the transposed projection, as stored on the device)."""
    base = np.uint64(splitmix64_int(seed))
    idx = np.arange(V * dim, dtype=np.uint64)
    u = splitmix64(base + idx)
    w = (((u >> np.uint64(32)) * np.uint64(255)) >> np.uint64(32)).astype(np.int64) - 127
    return w.reshape(dim, V)


def dense_features(indptr, bucket, count, V: int) -> np.ndarray:
    n = len(indptr) - 1
    F = np.zeros((n, V), dtype=np.int64)
    for c in range(n):
        F[c, bucket[indptr[c]:indptr[c + 1]]] = count[indptr[c]:indptr[c + 1]]
    return F


def embed(indptr, bucket, count, V: int, wt_int: np.ndarray, dtype: str = "f32") -> np.ndarray:
    F = dense_features(indptr, bucket, count, V)
    e = F @ wt_int.T                                   # int64 [n][dim]
    x = normalize_exact(e)
    if dtype == "f32":
        return x
    if dtype == "bf16":
        return f32_to_bf16_bits(x)
    if dtype == "f16":
        return x.astype(np.float16)
    raise ValueError(dtype)
