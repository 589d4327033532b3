// k_select.h — the two-pass scan's select: one 512-thread block takes one query's kept
// candidates from kernel 10's lists, finds its survivors, re-scores them exactly from the stored rows and
// writes the top-k.  A device function over the caller's LDS (SelLds); the select kernel is k_screen.hip's.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace sel {

using mfc::ord;
using mfc::unord;

struct Rec {  // the merge records of rfx/dist.py pack(): {f32 score, i32 pad, i64 row}
  float s;
  int pad;
  long long r;
};

template <int DT>
__device__ __forceinline__ float widen(uint16_t h) {
  if constexpr (DT == RFX_BF16)
    return __uint_as_float((uint32_t)h << 16);
  else
    return f16_to_f32(h);
}

constexpr int kSelCap = 2048;  // kept candidates per query held in LDS; more -> fallback (8 waves x 256)
constexpr int kSelK = 16;      // k <= kSelK (kernel 10 plans k <= 10)

#ifndef RFX_SEL_T
#define RFX_SEL_T(i)
#endif

// the select's LDS: survivor j's rank key (orderable fl32 of the exact f64 sum) << 32 | ~row — larger key =
// better under (score desc, row asc), so a rank is one 64-bit compare per survivor, no branches
struct SelLds {
  uint64_t skey[kSelCap];
  uint64_t res_key[64];                           // the answer, written out by one wave
  __attribute__((aligned(16))) float ca[kSelCap];  // screen score A of kept candidate i
  int crow[kSelCap];                              // its row
  int srow[kSelCap];                              // survivor j's row
  int n_c, n_sv, fail;
  float ak;
};

// one 16-B chunk's products added to acc in f64 (f32 products of bf16 / f16 values are exact; f32 values are
// multiplied in f64, also exact)
template <int DT>
__device__ __forceinline__ void chunk_dot(double& acc, const uint4& x, const uint4& y) {
  const uint32_t xx[4] = {x.x, x.y, x.z, x.w};
  const uint32_t yy[4] = {y.x, y.y, y.z, y.w};
  if constexpr (DT == RFX_F32) {
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += (double)__uint_as_float(xx[e]) * (double)__uint_as_float(yy[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint16_t xh = (uint16_t)(e & 1 ? xx[e >> 1] >> 16 : xx[e >> 1] & 0xffffu);
      const uint16_t yh = (uint16_t)(e & 1 ? yy[e >> 1] >> 16 : yy[e >> 1] & 0xffffu);
      acc += (double)(widen<DT>(xh) * widen<DT>(yh));
    }
  }
}

// Returns false (and sets the gate) when the query's survivors may be incomplete: nothing written.
template <int DT, int D>
__device__ __forceinline__ bool select_body(const float* __restrict__ cs, const int* __restrict__ cr,
                                            const uint32_t* __restrict__ drops, int64_t n_lists, int list_len,
                                            const float* __restrict__ qe2, const uint8_t* __restrict__ Q,
                                            const uint8_t* __restrict__ X, int k, int64_t row_offset,
                                            float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                            Rec* __restrict__ out_rec, uint32_t* __restrict__ gate,
                                            int* __restrict__ diag, int force, int64_t q, SelLds& sl) {
  // U1: candidate entries per thread per round (config 3: 512 lists x 10 = 5,120 = one round, rows
  // loaded with the scores, and the drops with them: one memory round trip instead of four).
  // The exact re-score: 16 lanes per survivor row (CPL 16-B chunks of the row per lane), U rows per
  // 16-lane group in flight: 8 waves x 4 groups x U = 96 rows per round (config 3: 94 survivors on
  // average, so one round, one memory latency)
  // rows and queries are read as 16-B chunks: chunk c of a row holds its bytes [16 c, 16 c + 16) (8 bf16 / f16
  // or 4 f32 elements); lane gl of a 16-lane group takes chunks gl + 16 i, i < CPL
  constexpr int RB = D * (DT == RFX_F32 ? 4 : 2);
  constexpr int NT = 512, NW = NT / 64, CPL = RB / 256, U = DT == RFX_F32 ? 2 : 3, U1 = 10, RPR = NW * 4 * U;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  RFX_SEL_T(0)
  if (tid == 0) {
    sl.n_c = sl.n_sv = sl.fail = 0;
    sl.ak = -__builtin_inff();
  }
  // the query's row chunks for the re-score (16-lane layout below), loaded with everything else
  const int gl = lane & 15, grp = w * 4 + (lane >> 4);
  uint4 yq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) yq[c] = *(const uint4*)(Q + q * RB + (gl + 16 * c) * 16);
  __syncthreads();
  // 1. compact the kept candidates (the scan wrote -inf for empty slots and dropped entries)
  const int64_t n = n_lists * list_len;
  const float* qs = cs + q * n;
  const int* qr = cr + q * n;
  const uint32_t d0 = tid < n_lists ? drops[q * n_lists + tid] : 0u;  // step 3's, loaded now
  for (int64_t b = tid; b < n; b += (int64_t)NT * U1) {
    float s[U1];
    int r[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const bool in = b + u * NT < n;
      s[u] = in ? qs[b + u * NT] : -__builtin_inff();
      r[u] = in ? qr[b + u * NT] : 0;
    }
#pragma unroll
    for (int u = 0; u < U1; ++u)
      if (s[u] != -__builtin_inff()) {
        const int i = atomicAdd(&sl.n_c, 1);
        if (i < kSelCap) {
          sl.ca[i] = s[u];
          sl.crow[i] = r[u];
        }
      }
  }
  __syncthreads();
  RFX_SEL_T(1)
  const int nc = sl.n_c;
  if (nc > kSelCap || force) sl.fail = 1;
  const int ncl = nc < kSelCap ? nc : kSelCap;
  // 2. a_k = the k-th best A (with multiplicity): the value v with #{> v} < k <= #{>= v}.  Every
  // candidate counts the others with 16-B broadcast reads (4 per read; the tail padded with -inf,
  // which counts for nothing).  Measured faster than extracting each wave's k best by k rounds of a
  // DPP wave max (1.96 against 4.72 us at the 8-GPU shard, ~108 candidates per query: those rounds
  // are a serial dependency chain).
  if (tid < 3 && ncl + tid < kSelCap) sl.ca[ncl + tid] = -__builtin_inff();
  __syncthreads();
  {
    const float4* ca4 = (const float4*)sl.ca;
    const int n4 = (ncl + 3) >> 2;
    for (int i = tid; i < ncl; i += NT) {
      const float si = sl.ca[i];
      int gt = 0, ge = 0;
#pragma unroll 8
      for (int j = 0; j < n4; ++j) {
        const float4 v = ca4[j];
        gt += (v.x > si) + (v.y > si) + (v.z > si) + (v.w > si);
        ge += (v.x >= si) + (v.y >= si) + (v.z >= si) + (v.w >= si);
      }
      if (gt < k && ge >= k) sl.ak = si;  // every writer writes the same value
    }
  }
  __syncthreads();
  RFX_SEL_T(2)
  const float e2 = qe2[q];
  const float t = ncl >= k ? sl.ak - e2 : -__builtin_inff();
  const uint32_t ot = ord(t);
  // 3. a row dropped at or above t could be a survivor the lists lost: fallback
  if (d0 && d0 >= ot) sl.fail = 1;
  for (int64_t j = tid + NT; j < n_lists; j += NT) {
    const uint32_t d = drops[q * n_lists + j];
    if (d && d >= ot) sl.fail = 1;
  }
  for (int i = tid; i < ncl; i += NT)
    if (sl.ca[i] >= t) sl.srow[atomicAdd(&sl.n_sv, 1)] = sl.crow[i];
  __syncthreads();
  RFX_SEL_T(3)
  if (sl.fail) {
    if (tid == 0) __hip_atomic_store(gate, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (diag && tid == 0) {
      __hip_atomic_store(diag + q * 2, nc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(diag + q * 2 + 1, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return false;  // the exact fallback answers this query
  }
  const int ns = sl.n_sv;
  // 4. exact re-score: the 16 lanes of a group hold chunks gl + 16 c of the row (8 elements each); f32
  // products of bf16 / f16 values are exact, their sum is taken in f64 (the oracle's f64 dot up to
  // f64 rounding), rounded once to f32
  for (int j0 = grp; j0 < ns; j0 += RPR) {
    uint4 xv[U][CPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * NW * 4;
      const int64_t row = j < ns ? (int64_t)sl.srow[j] : (int64_t)sl.srow[0];
#pragma unroll
      for (int c = 0; c < CPL; ++c) xv[u][c] = *(const uint4*)(X + row * RB + (gl + 16 * c) * 16);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < CPL; ++c) chunk_dot<DT>(acc, xv[u][c], yq[c]);
      acc = row16_sum_f64(acc);  // within the 16-lane group (DPP; lane 0's sum = the xor butterfly's)
      const int j = j0 + u * NW * 4;
      if (gl == 0 && j < ns) sl.skey[j] = ((uint64_t)ord((float)acc) << 32) | (uint32_t)(~(uint32_t)sl.srow[j]);
    }
  }
  __syncthreads();
  RFX_SEL_T(4)
  // 5. top-k of the survivors by (exact score desc, row asc) with the exact score rounded to f32 first
  // (the order every merge of f32 scores keeps: a sharded store's gathered merge, kernel 11); NaN
  // (cannot occur for live rows) last.  The k best land in LDS; one wave writes them out.
  for (int j = tid; j < ns; j += NT) {
    const uint64_t kj = sl.skey[j];
    int rank = 0;
#pragma unroll 8
    for (int i = 0; i < ns; ++i) rank += sl.skey[i] > kj ? 1 : 0;
    if (rank < k) sl.res_key[rank] = kj;
  }
  RFX_SEL_T(6)
  __syncthreads();
  if (tid < k) {
    const bool ok = tid < ns;  // (survivors are live rows: never NaN)
    const uint64_t kk = ok ? sl.res_key[tid] : 0ull;
    const float sf = ok ? unord((uint32_t)(kk >> 32)) : -__builtin_inff();
    const long long rr = ok ? (long long)(int)(~(uint32_t)kk) + row_offset : -1;
    if (out_rec) {
      out_rec[q * k + tid] = Rec{sf, 0, rr};
    } else {
      out_s[q * k + tid] = sf;
      out_r[q * k + tid] = rr;
    }
  }
  if (diag && tid == 0) {
    __hip_atomic_store(diag + q * 2, nc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(diag + q * 2 + 1, ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RFX_SEL_T(5)
  return true;
}

}  // namespace sel
}  // namespace rfx
