// k_scan_valu.h — the VALU fused scan + top-k kernel template (nq <= 8 per slice) and the device
// merge routines it shares with the merge kernels.  Instantiated per index dtype in valu_f32.hip,
// valu_bf16.hip and valu_f16.hip (three translation units, compiled in parallel); the launchers,
// plan and merge kernels are in k_scan_valu.hip.
//
// Path: query×corpus inner-product scan + per-query top-k (the retrieval half of
// GeminiRag.ask_stream, backend/app/services/gemini_rag.py:517-551, which the reference runs
// remotely).
#pragma once
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {

// ---------------------------------------------------------------------------------------
// VALU fused scan + top-k (nq <= 8 per launch slice).
//   X      : [nrows][D] dtype DT
//   Qf     : [nq][D] f32 (exact widening of the index-dtype queries)
//   output : cand_s/cand_r [nq][n_lists][K], n_lists = gridDim.x (the 4 wave lists merged per block)
// Algorithmic bytes per row: D * esz (the row is read once for all NQT queries).
// ---------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ float elem(const uint4& v, int e) {
  const uint32_t w = (&v.x)[DT == RFX_F32 ? e : (e >> 1)];
  if constexpr (DT == RFX_F32) {
    return __uint_as_float(w);
  } else if constexpr (DT == RFX_BF16) {
    return (e & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
  } else {
    return f16_to_f32((e & 1) ? (uint16_t)(w >> 16) : (uint16_t)(w & 0xffffu));
  }
}

struct MergeRec {  // 16 B; the layout of rfx/dist.py pack(): int64(score bits) + int64 row
  float s;
  int pad;
  long long r;
};

template <bool R64>
struct FlatSrc {
  const float* cs;
  const void* cr;
  int64_t n;  // candidates per query
  __device__ __forceinline__ void get(int64_t q, int64_t i, float& s, long long& r) const {
    s = cs[q * n + i];
    if constexpr (R64)
      r = ((const long long*)cr)[q * n + i];
    else
      r = (long long)((const int*)cr)[q * n + i];
  }
};
struct GatheredSrc {
  const MergeRec* rec;
  int64_t nq;
  int k;  // entries per rank (= list_len)
  int64_t n;
  __device__ __forceinline__ void get(int64_t q, int64_t i, float& s, long long& r) const {
    const int ii = (int)i;  // n_cand < 2^31 (host check)
    const int64_t rank = ii / k, e = ii - (ii / k) * k;
    const MergeRec m = rec[(rank * nq + q) * k + e];
    s = m.s;
    r = m.r;
  }
};

constexpr long long kNoRow = 0x7fffffffffffffffll;

// [nq][n] candidates read with agent-scope loads (sc1): the one-launch search's last block reads
// what the other blocks of its slice stored the same way during the launch.
struct AgentSrc {
  const float* cs;
  const int* cr;
  int64_t n;
  __device__ __forceinline__ void get(int64_t q, int64_t i, float& s, long long& r) const {
    s = __uint_as_float(__hip_atomic_load((const uint32_t*)cs + q * n + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    r = (long long)__hip_atomic_load(cr + q * n + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// One query's candidates staged in LDS by the fused search's last block (up to kFusedLdsCand).
constexpr int kFusedLdsCand = 4096;
struct LdsSrc {
  const float* s;
  const int* r;
  int64_t n;
  __device__ __forceinline__ void get(int64_t, int64_t i, float& sc, long long& rr) const {
    sc = s[i];
    rr = (long long)r[i];
  }
};

// FUSED (the whole search in one launch, rfx_search on a VALU plan): the queries are read in the
// index dtype and widened here (no widen kernel), and the last block of each query slice to finish
// (agent-scope release/acquire on a per-slice counter) merges the slice's candidates into the final
// top-k (no merge launch), then returns the launch state (bounds, counter) to zero for the next
// search on the same stream.  `Qf` is then the raw [nq][D] query buffer in dtype DT.
struct FusedOut {
  uint32_t* ctr;  // [q_slices] arrival counters (zero on entry, left zero)
  int k_out;
  float* out_s;
  int64_t* out_r;
  // the two-pass scan's fallback (k_screen_valu.hip): run only when the screen set this word, and the
  // final top-k re-scored by the two-pass rule (Rescore above; rows = the scan's X, queries = Qf)
  const uint32_t* gate = nullptr;
};

// The score rule of every search (round 5: one rule for every plan): a returned score is fl32(exact
// dot), the f64 sum of the exact products rounded once, and the order is (that f32 score desc, row asc)
// — what kernel 10's select and kernel 11's last block return.  The exact scans (f32 accumulation:
// kernels 1-3, 6, 8, 9, VALU) pick their final top-k by their own sums and that top-k is then
// re-scored and re-ordered by the same rule (`Rescore`: here in the one-launch VALU search, and in the
// merge of every other exact plan and of the two-pass scan's gated fallback), so an answer's bits do
// not depend on which path a query (or a shard of a sharded store) took.  (The SET can differ from the
// two-pass scan's only where two rows' exact scores lie within the f32 accumulation error of each other
// at the k-th place)
// (struct Rescore: rfx_kernels.h)

__device__ __forceinline__ float elem_rt(const void* p, int64_t i, int dtype) {
  if (dtype == RFX_F32) return ((const float*)p)[i];
  const uint16_t h = ((const uint16_t*)p)[i];
  return dtype == RFX_BF16 ? bf16_to_f32(h) : f16_to_f32(h);
}

// Block-wide (any block size that is a multiple of 64, k_out <= 64): the k_out entries just written
// for query q (out_s / out_r, or out_rec; the merge added row_offset to the rows in both forms, so the
// row of X is row - row_offset either way) re-scored and re-ordered by the rule above.  The caller's
// writes are read back with agent-scope loads after a barrier.
__device__ __forceinline__ void rescore_final(const Rescore& rs, int64_t q, int k_out, int64_t row_offset,
                                              float* out_s, int64_t* out_r, MergeRec* out_rec) {
  __shared__ float rs_s[64];
  __shared__ long long rs_r[64];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tid = threadIdx.x, nt = blockDim.x, gl = tid & 7;
  for (int e0 = 0; e0 < k_out; e0 += nt / 8) {
    const int e = e0 + (tid >> 3);
    long long row = -1;
    if (e < k_out) {
      const int64_t o = q * k_out + e;
      row = out_rec ? (long long)__hip_atomic_load((const unsigned long long*)&out_rec[o].r, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                    : (long long)__hip_atomic_load((const unsigned long long*)out_r + o, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    // an entry whose row lies outside this index's [row_offset, row_offset + rows) is padding (ADVICE r5:
    // rfx_rescore_topk takes hand-assembled answers; a merged multi-shard row must not index past X)
    if (row < row_offset || row - row_offset >= rs.rows) row = -1;
    double acc = 0.0;
    if (row >= 0) {
      const int64_t xr = (row - row_offset) * rs.D, qr = q * rs.D;
      for (int c = gl; c < rs.D; c += 8)
        acc += (double)elem_rt(rs.X, xr + c, rs.dtype) * (double)elem_rt(rs.Q, qr + c, rs.dtype);
    }
#pragma unroll
    for (int off = 4; off; off >>= 1) acc += __shfl_xor(acc, off);
    if (gl == 0 && e < k_out) {
      rs_s[e] = row >= 0 ? (float)acc : -__builtin_inff();
      rs_r[e] = row;
    }
  }
  __syncthreads();
  if (tid < k_out) {
    const float s = rs_s[tid];
    const long long r = rs_r[tid];
    int n_valid = 0;
    for (int f = 0; f < k_out; ++f) n_valid += rs_r[f] >= 0;
    if (r >= 0) {
      // rank among the valid entries (a repeated entry ranks after its earlier copy: every rank is taken once)
      int rank = 0;
      for (int f = 0; f < k_out; ++f)
        rank += rs_r[f] >= 0 && (better64(rs_s[f], rs_r[f], s, r) || (f < tid && rs_s[f] == s && rs_r[f] == r));
      const int64_t o = q * k_out + rank;
      if (out_rec) {
        out_rec[o] = MergeRec{s, 0, r};
      } else {
        out_s[o] = s;
        out_r[o] = r;
      }
    }
    if (tid >= n_valid) {  // the padding goes last, whatever positions it held
      const int64_t o = q * k_out + tid;
      if (out_rec) {
        out_rec[o] = MergeRec{-__builtin_inff(), 0, -1};
      } else {
        out_s[o] = -__builtin_inff();
        out_r[o] = -1;
      }
    }
  }
  __syncthreads();
}

template <int DT>
__device__ __forceinline__ float query_elem(const void* Q, int64_t i) {
  if constexpr (DT == RFX_F32)
    return ((const float*)Q)[i];
  else if constexpr (DT == RFX_BF16)
    return bf16_to_f32(((const uint16_t*)Q)[i]);
  else
    return f16_to_f32(((const uint16_t*)Q)[i]);
}

template <int K, bool R64, int NW, bool SORTED, class Src>
__device__ __forceinline__ void merge_one(const Src& src, int64_t q, int list_len, int k_out, int64_t row_offset,
                                          float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                          MergeRec* __restrict__ out_rec);

// The scan's body, a device function over VIRTUAL blocks: vblk (< nvb) stands for blockIdx.x (its rows,
// its candidate list) and the FUSED arrival counts nvb virtual blocks, so the final merge runs once
// every virtual block has finished, whichever workgroups ran them.  The kernel below runs one virtual
// block per workgroup (vblk = blockIdx.x); kernel 11 (k_screen_valu.hip) runs its exact fallback inside
// its own launch by having its workgroups CLAIM virtual blocks from a counter (round 5): the fallback
// completes whichever of them run, so it needs no co-residency of the grid.
template <int DT, int NQT, int K, int VPL, bool FUSED>
__device__ __forceinline__ void scan_valu_body(const uint8_t* __restrict__ X, int nrows, int D,
                                               const void* __restrict__ Qf, int nq, int rows_per_wave,
                                               float* __restrict__ cand_s, int* __restrict__ cand_r,
                                               int n_lists, const uint32_t* __restrict__ mask,
                                               uint32_t* __restrict__ tau, const FusedOut& fo, int vblk, int nvb) {
  constexpr int ESZ = DT == RFX_F32 ? 4 : 2;
  constexpr int EPV = 16 / ESZ;
  extern __shared__ __attribute__((aligned(16))) float q_lds[];  // [NQT][D]
  const int tid = threadIdx.x;
  const int lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int q0 = blockIdx.y * NQT;
  const int nqt = min(NQT, nq - q0);
  const int VPR = D * ESZ / 16;
  const int64_t RB = (int64_t)D * ESZ;
  const int wave_g = vblk * 4 + (tid >> 6);
  const int wb = (int)min((int64_t)wave_g * rows_per_wave, (int64_t)nrows);
  const int we = (int)min((int64_t)wb + rows_per_wave, (int64_t)nrows);

  WaveList<K> L[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) L[qi].init();

  float cand[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) cand[qi] = 0.f;
  float qr[NQT == 1 ? VPL * EPV : 1];  // NQT == 1: the lane's query elements (filled below)

  // Row stream, software-pipelined: iteration t covers rows wb + 64 (t >> 4) + 4 (t & 15) + g (one
  // row per 16-lane group); the loads of iteration t + 1 are in flight while iteration t computes,
  // so a wave never drains its loads at a loop back-edge (with one or two waves per SIMD nothing
  // else hides that latency).  Rows past `we` re-read row wb (cache hits) and are never offered.
  auto load_row = [&](int t, uint4 (&v)[VPL]) {
    const int row = wb + 64 * (t >> 4) + 4 * (t & 15) + g;
    const uint8_t* rp = X + (int64_t)(row < we ? row : wb) * RB;
    // unconditional loads (clamped address, zeroed by a select): no branch around a load, so
    // the compiler counts vmcnt per buffer instead of draining at every branch join
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vv = j + 16 * i;
      const uint4 x = *(const uint4*)(rp + (int64_t)(vv < VPR ? vv : VPR - 1) * 16);
      const uint32_t m = vv < VPR ? 0xffffffffu : 0u;  // AND, not a select (which becomes a branch)
      v[i] = make_uint4(x.x & m, x.y & m, x.z & m, x.w & m);
    }
  };
  auto score_row = [&](int it, const uint4 (&v)[VPL]) {
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        if (16 * i >= VPR) continue;
#pragma unroll
        for (int e = 0; e < EPV; ++e) {
          float qv;
          if constexpr (NQT == 1)
            qv = qr[i * EPV + e];
          else
            qv = (j + 16 * i < VPR) ? q_lds[qi * D + (j + 16 * i) * EPV + e] : 0.f;
          acc = fmaf(elem<DT>(v[i], e), qv, acc);
        }
      }
      acc = row16_sum(acc);
      if (j == it) cand[qi] = acc;
    }
  };
  // iterations: 4 rows each, rounded up to the loop's unroll of 4 (not to a whole 64-row chunk: a
  // wave's last chunk is usually partial, and iterations past its rows only re-read row wb)
  const int T = we > wb ? (we - wb + 15) / 16 * 4 : 0;
  // three iterations in flight ahead of the one being scored (48 KB per wave at d 768 f32): one
  // wave per SIMD has nothing else to hide the loads' latency
  uint4 va[VPL], vb[VPL], vc[VPL], vd[VPL];
  if constexpr (NQT == 1) {
    // one query: each lane loads its own query elements straight into registers (every block
    // reads the same d values: L2 hits), before the row loads, so waiting for them never waits
    // for a row; clamped index + AND mask, no branch around a load.  No LDS, no barrier.
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = j + 16 * i;
      const int vv = v < VPR ? v : VPR - 1;
      const uint32_t m = v < VPR ? 0xffffffffu : 0u;
      if constexpr (FUSED) {  // the query in the index dtype: the row's own 16-B layout
        const uint4 u = *(const uint4*)((const uint8_t*)Qf + (int64_t)q0 * RB + (int64_t)vv * 16);
#pragma unroll
        for (int e = 0; e < EPV; ++e) qr[i * EPV + e] = __uint_as_float(__float_as_uint(elem<DT>(u, e)) & m);
      } else {  // widened f32 queries: EPV floats per 16 B of row
        const float* qf = (const float*)Qf + (int64_t)q0 * D + (int64_t)vv * EPV;
#pragma unroll
        for (int h = 0; h < EPV / 4; ++h) {
          const uint4 u = *(const uint4*)(qf + 4 * h);
          qr[i * EPV + 4 * h + 0] = __uint_as_float(u.x & m);
          qr[i * EPV + 4 * h + 1] = __uint_as_float(u.y & m);
          qr[i * EPV + 4 * h + 2] = __uint_as_float(u.z & m);
          qr[i * EPV + 4 * h + 3] = __uint_as_float(u.w & m);
        }
      }
    }
  }
  if (T > 0) {  // the first rows are in flight while the query is staged
    load_row(0, va);
    load_row(1, vb);
    load_row(2, vc);
  }
  if constexpr (NQT != 1) {
    for (int i = tid; i < NQT * D; i += 256) {
      const int qi = i / D;
      const int64_t src = (int64_t)(q0 + qi) * D + (i - qi * D);
      q_lds[i] = qi >= nqt ? 0.f : FUSED ? query_elem<DT>(Qf, src) : ((const float*)Qf)[src];
    }
    __syncthreads();
  }

  // Loads past the last iteration read row wb again (load_row clamps): unconditional, so no branch
  // around a load.
  for (int t = 0; t < T; t += 4) {
    load_row(t + 3, vd);  // T is a multiple of 4: t + 3 < T
    score_row(t & 15, va);
    load_row(t + 4, va);
    score_row((t + 1) & 15, vb);
    load_row(t + 5, vb);
    score_row((t + 2) & 15, vc);
    load_row(t + 6, vc);
    score_row((t + 3) & 15, vd);
    if (((t + 4) & 15) == 0 || t + 4 >= T) {  // chunk done (or the last, partial one): offer it
      // lanes j of a partial chunk past its last iteration hold rows >= we: never offered
      const int crow = wb + 64 * (t >> 4) + j * 4 + g;
      // metadata filter: rows whose mask bit is clear are never offered
      const bool ok = crow < we && (mask == nullptr || row_allowed(mask, crow));
#pragma unroll
      for (int qi = 0; qi < NQT; ++qi) L[qi].offer(cand[qi], crow, ok);
    }
  }

  // block-level merge: the 4 wave lists of a query -> one list per block (4x fewer candidates
  // for the merge kernel, which dominates single-query latency); wave w merges queries w, w+4, ..
  __shared__ float ms[4][NQT][K];
  __shared__ int mr[4][NQT][K];
  const int w = tid >> 6;
  // the queries' running bounds as they stand now, read before the LDS merge so the load's latency
  // hides behind it (any value read is a valid bound)
  uint32_t seen[(NQT + 3) / 4];
#pragma unroll
  for (int u = 0; u < (NQT + 3) / 4; ++u) {
    const int qi = w + 4 * u;
    seen[u] = tau && qi < nqt ? __hip_atomic_load(tau + q0 + qi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  }
  if (lane < K) {
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      ms[w][qi][lane] = L[qi].ls;
      mr[w][qi][lane] = L[qi].lr;
    }
  }
  __syncthreads();
  for (int qi = w; qi < nqt; qi += 4) {
    WaveList<K> M;
    M.init();
#pragma unroll
    for (int src = 0; src < 4; ++src) {
      const bool v = lane < K;
      M.offer(v ? ms[src][qi][lane] : -__builtin_inff(), v ? mr[src][qi][lane] : kEmptyRow,
              v && mr[src][qi][lane] != kEmptyRow);
    }
    // cross-block pruning: every block's K-th best is a lower bound of the query's K-th best
    // (>= its k-th best), so entries below the running max of those bounds can never be
    // returned; write them as empty (the merge skips them without an insert).
    uint32_t bound = 0u;
    if (tau) {
      const float kth = readlane_f(M.ls, K - 1);
      const uint32_t mine = kth > -__builtin_inff() ? ord_f32(kth) : 0u;
      // publish without waiting for the old value (no-return atomic): its round trip overlaps the
      // candidate stores instead of preceding them
      if (lane == 0) __hip_atomic_fetch_max(tau + q0 + qi, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bound = max(seen[(qi - w) / 4], mine);
    }
    if (lane < K) {
      const int64_t o = ((int64_t)(q0 + qi) * n_lists + vblk) * K + lane;
      const bool keep = M.lr != kEmptyRow && ord_f32(M.ls) >= bound;
      const float cs_v = keep ? M.ls : -__builtin_inff();
      const int cr_v = keep ? M.lr : kEmptyRow;
      if constexpr (FUSED) {  // agent-coherent stores (sc1): the slice's last block reads them
        __hip_atomic_store((uint32_t*)cand_s + o, __float_as_uint(cs_v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cand_r + o, cr_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        cand_s[o] = cs_v;
        cand_r[o] = cr_v;
      }
    }
  }
  if constexpr (FUSED) {
    // Hand-off without cache maintenance: the candidates went out as agent-scope (sc1) stores, so
    // once every lane's stores are acknowledged (vmcnt 0) they are visible at the device's
    // coherence point; the arrival counter is an agent-scope atomic, and the last block reads
    // the candidates with agent-scope loads.  (A release/acquire fence pair here writes back and
    // invalidates the XCD's whole L2 in every block: measured 1.6x slower at config 2.)
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint32_t old =
          __hip_atomic_fetch_add(fo.ctr + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == (uint32_t)nvb - 1u;
    }
    __syncthreads();
    // (readfirstlane: a uniform branch for the compiler, so a caller's loop around this body keeps its
    // barriers in uniform control flow; kernel 11's claim loop below hung without it, round 5)
    if (!__builtin_amdgcn_readfirstlane(last)) return;
    const int64_t n = (int64_t)n_lists * K;
    if (n <= kFusedLdsCand) {
      // Bulk copy first: every candidate of the query is loaded with all loads in flight (one
      // memory latency per 8 per thread) into LDS, then merged from there.  Merging straight from
      // memory walks each sorted list with one dependent agent-scope load per entry.
      __shared__ float bs[kFusedLdsCand];
      __shared__ int br[kFusedLdsCand];
      const LdsSrc lsrc{bs, br, n};
      for (int qi = 0; qi < nqt; ++qi) {
        const int64_t qo = (int64_t)(q0 + qi) * n;
        for (int base = 0; base < (int)n; base += 256 * 8) {
          uint32_t sv[8];
          int rv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = base + u * 256 + tid;
            if (i < (int)n) {
              sv[u] = __hip_atomic_load((const uint32_t*)cand_s + qo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              rv[u] = __hip_atomic_load(cand_r + qo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = base + u * 256 + tid;
            if (i < (int)n) {
              bs[i] = __uint_as_float(sv[u]);
              br[i] = rv[u];
            }
          }
        }
        __syncthreads();
        merge_one<K, false, 4, true>(lsrc, q0 + qi, K, fo.k_out, 0, fo.out_s, fo.out_r, nullptr);
        __syncthreads();
        rescore_final(Rescore{X, Qf, D, DT, (int64_t)nrows}, q0 + qi, fo.k_out, 0, fo.out_s, fo.out_r, nullptr);
      }
    } else {
      const AgentSrc src{cand_s, cand_r, n};
      for (int qi = 0; qi < nqt; ++qi) {
        merge_one<K, false, 4, true>(src, q0 + qi, K, fo.k_out, 0, fo.out_s, fo.out_r, nullptr);
        __syncthreads();
        rescore_final(Rescore{X, Qf, D, DT, (int64_t)nrows}, q0 + qi, fo.k_out, 0, fo.out_s, fo.out_r, nullptr);
      }
    }
    if (tid < nqt && tau) tau[q0 + tid] = 0u;  // every block's bound updates precede its arrival
    if (tid == 0) fo.ctr[blockIdx.y] = 0u;
  }
}

template <int DT, int NQT, int K, int VPL, bool FUSED>
__global__ __launch_bounds__(256) void scan_valu_kernel(const uint8_t* __restrict__ X, int nrows, int D,
                                                        const void* __restrict__ Qf, int nq,
                                                        int rows_per_wave, float* __restrict__ cand_s,
                                                        int* __restrict__ cand_r, int n_lists,
                                                        const uint32_t* __restrict__ mask,
                                                        uint32_t* __restrict__ tau, FusedOut fo) {
  if constexpr (FUSED)  // gated (the two-pass scan's fallback): the whole grid returns together
    if (fo.gate && __hip_atomic_load(fo.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  scan_valu_body<DT, NQT, K, VPL, FUSED>(X, nrows, D, Qf, nq, rows_per_wave, cand_s, cand_r, n_lists, mask, tau, fo,
                                         (int)blockIdx.x, (int)gridDim.x);
}

// K values instantiated for the scan; runtime k is rounded up to one of these and only the
// first k entries of each list are used by the merge (lists are sorted).
#define RFX_VALU_K_LIST(X_) X_(4) X_(16) X_(64)

template <int DT, int NQT, int K>
inline int launch_valu_vpl(int vpl, dim3 grid, size_t lds, hipStream_t st, const uint8_t* X, int nrows,
                           int D, const void* Qf, int nq, int rpw, float* cs, int* cr, int n_lists,
                           const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
#define RFX_L(V)                                                                                       \
  if (vpl <= V) {                                                                                      \
    if (fo.ctr)                                                                                        \
      hipLaunchKernelGGL((scan_valu_kernel<DT, NQT, K, V, true>), grid, dim3(256), lds, st, X, nrows, D, \
                         Qf, nq, rpw, cs, cr, n_lists, mask, tau, fo);                                 \
    else                                                                                               \
      hipLaunchKernelGGL((scan_valu_kernel<DT, NQT, K, V, false>), grid, dim3(256), lds, st, X, nrows,   \
                         D, Qf, nq, rpw, cs, cr, n_lists, mask, tau, fo);                              \
    return 0;                                                                                          \
  }
  RFX_L(4) RFX_L(8) RFX_L(12) RFX_L(16)
#undef RFX_L
  return -1;
}

template <int DT, int NQT>
inline int launch_valu_k(int kk, int vpl, dim3 grid, size_t lds, hipStream_t st, const uint8_t* X,
                         int nrows, int D, const void* Qf, int nq, int rpw, float* cs, int* cr,
                         int n_lists, const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
#define RFX_K(KV) \
  if (kk == KV) return launch_valu_vpl<DT, NQT, KV>(vpl, grid, lds, st, X, nrows, D, Qf, nq, rpw, cs, cr, n_lists, mask, tau, fo);
  RFX_VALU_K_LIST(RFX_K)
#undef RFX_K
  return -1;
}

// ---------------------------------------------------------------------------------------
// Top-k merge: one 512-thread block per query.  The candidates of a query are groups of
// `list_len` (the scan kernels' sorted partial lists, best first; list_len = 1: no structure).
//   bound:  with list_len >= k, T = max over lists of the min of the list's first k entries (a
//           lower bound of the query's k-th best); the wave lists admit only scores >= T.
//   pass:   the 8 waves fold every candidate (one ballot per 64; below T nothing is inserted);
//   final:  rank_merge of the 8 wave lists.
// Sources: flat [nq][n_cand] (score, row) arrays, or the all-gathered per-rank records of the
// multi-GPU path ([world][nq][k] of {f32 score, pad, i64 row}).
// ---------------------------------------------------------------------------------------

// Fold candidates i = base + (p * NW * 64) + lane, p < P, of one query into the wave list.  All P
// loads are issued before the first offer, so a chunk costs one memory latency, not P.
template <int K, bool R64, int P, int NW, class Src>
__device__ __forceinline__ void merge_chunk(const Src& src, int64_t q, int64_t base, int64_t n, int lane,
                                            WaveList64<K>& L) {
  float sc[P];
  long long rr[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t i = base + (int64_t)p * NW * 64 + lane;
    sc[p] = -__builtin_inff();
    rr[p] = kNoRow;
    if (i < n) src.get(q, i, sc[p], rr[p]);  // (n < 2^31)
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    // empty slots of partial lists carry a sentinel row: never valid candidates
    const bool live = rr[p] >= 0 && rr[p] != kNoRow && (R64 || rr[p] != (long long)kEmptyRow);
    L.offer(sc[p], rr[p], live);
  }
}

// Block-wide merge of M sorted lists of K (best first, padded with (-inf, kNoRow)) in LDS into the
// top-K list `dst` (pre-filled with padding by the caller): every thread takes candidates and
// computes their rank as its index plus, for each other list, the number of entries better than
// it (binary search).  The ranks of distinct (score, row) pairs are distinct, so each of the K
// best lands in its own slot.  O(M log K) per candidate, no serial chain.
template <int K, int M>
__device__ __forceinline__ void rank_merge(const float (*ls)[K], const long long (*lr)[K], float* dst_s,
                                           long long* dst_r) {
  for (int t = threadIdx.x; t < M * K; t += blockDim.x) {
    const int m = t / K, e = t - (t / K) * K;
    const float s = ls[m][e];
    const long long r = lr[m][e];
    if (r == kNoRow) continue;
    int rank = e;
    for (int mm = 0; mm < M && rank < K; ++mm) {
      if (mm == m) continue;
      int lo = 0, hi = K;  // first entry of list mm that is not better than (s, r)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (better64(ls[mm][mid], lr[mm][mid], s, r))
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < K) {
      dst_s[rank] = s;
      dst_r[rank] = r;
    }
  }
}

// One query's merge by a block of NW waves (the merge kernel: NW = 8; the fused single-launch
// VALU search's last block: NW = 4).
// SORTED: each list of list_len entries is sorted best first with its empty slots at the tail
// (what every scan kernel writes, and the per-rank records of the multi-GPU path).  Then a list is
// read only as far as its entries can still be admitted — the heads bound usually rejects a whole
// list at its first entry — and the list-bound pass (every list's first k entries) is skipped.
template <int K, bool R64, int NW, bool SORTED, class Src>
__device__ __forceinline__ void merge_one(const Src& src, int64_t q, int list_len, int k_out, int64_t row_offset,
                                          float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                          MergeRec* __restrict__ out_rec) {
  constexpr int NT = NW * 64;
  // rows 0..NW-1: wave lists, row NW: the final list
  __shared__ float ls_lds[NW + 1][K];
  __shared__ long long lr_lds[NW + 1][K];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t n = src.n;
  constexpr int P = 8;  // chunk: 8 * NT candidates per block
  if (tid < K) {
    ls_lds[NW][tid] = -__builtin_inff();
    lr_lds[NW][tid] = kNoRow;
  }
  // ---- bound: with lists of list_len >= k_out entries, the minimum of a list's first k_out
  // entries is a lower bound of the query's k_out-th best (that list alone holds k_out candidates
  // at or above it; for the scan's sorted lists it is the k_out-th entry), so the max over lists
  // T only admits what can still be returned — exact whether or not the lists are sorted ----
  WaveList64<K> L;
  L.init();
  __shared__ uint32_t tb;
  // ---- heads bound: the first entries of up to 512 lists are distinct candidates, so the k_out-th
  // best of them is a lower bound of the query's k_out-th best.  Each live head counts the heads at
  // or above it (broadcast LDS reads); T_heads = the best head with >= k_out heads at or above it.
  // Far tighter than the list bound when there are many short lists (config 2: 391 lists of 16,
  // the admitted candidates drop from ~3,200 to tens) ----
  __shared__ uint4 hk4[128];
  uint32_t* hk = (uint32_t*)hk4;
  const int64_t n_heads64 = n / list_len;
  const int nh = (int)(n_heads64 < 512 ? n_heads64 : 512);
  uint32_t mine[512 / NT];
  if (tid == 0) tb = 0u;
#pragma unroll
  for (int u = 0; u < 512 / NT; ++u) {
    const int h = tid + u * NT;
    mine[u] = 0u;
    if (h < nh) {
      float hs;
      long long hr;
      src.get(q, (int64_t)h * list_len, hs, hr);
      const bool live = hr >= 0 && hr != kNoRow && (R64 || hr != (long long)kEmptyRow);
      mine[u] = live ? ord_f32(hs) : 0u;
    }
  }
  uint32_t m = 0u;  // list bound (below), reduced after the barrier
  if (!SORTED && list_len > 1 && list_len >= k_out) {
    for (int64_t j = tid; j < n / list_len; j += NT) {
      uint32_t mj = 0xffffffffu;  // min over the list's first k_out entries (sorted or not)
      for (int e0 = 0; e0 < k_out; e0 += 8) {  // 8 independent loads in flight per round
        float sc[8];
        long long rr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sc[u] = __builtin_inff();
          rr[u] = 0;
          if (e0 + u < k_out) src.get(q, j * list_len + e0 + u, sc[u], rr[u]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool live = rr[u] >= 0 && rr[u] != kNoRow && (R64 || rr[u] != (long long)kEmptyRow);
          mj = min(mj, live ? ord_f32(sc[u]) : 0u);
        }
      }
      m = max(m, mj);
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  }
#pragma unroll
  for (int u = 0; u < 512 / NT; ++u) hk[tid + u * NT] = mine[u];  // after the list pass: loads overlap
  __syncthreads();
  if (nh >= k_out) {
    uint32_t cand = 0u;
#pragma unroll
    for (int u = 0; u < 512 / NT; ++u) {
      if (mine[u]) {
        int c = 0;
        for (int i = 0; i < (nh + 3) / 4; ++i) {
          const uint4 v = hk4[i];
          c += (v.x >= mine[u]) + (v.y >= mine[u]) + (v.z >= mine[u]) + (v.w >= mine[u]);
        }
        if (c >= k_out) cand = max(cand, mine[u]);
      }
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) cand = max(cand, (uint32_t)__shfl_xor((int)cand, off));
    if (lane == 0 && cand) atomicMax(&tb, cand);
  }
  if (lane == 0 && m) atomicMax(&tb, m);
  __syncthreads();
  if (tb) {
    const uint32_t u = tb & 0x80000000u ? tb & 0x7fffffffu : ~tb;  // inverse of ord_f32
    L.init_above(__uint_as_float(u), kNoRow);                      // admits score >= T
  }
  if constexpr (SORTED) {
    // lane walks list lb + lane while its entries still beat the wave list's admission bound
    // (wave-uniform; it only rises): a sorted list's later entries cannot do better
    const int64_t nl = n / list_len;
    for (int64_t lb = (int64_t)w * 64; lb < nl; lb += NT) {
      const int64_t li = lb + lane;
      bool alive = li < nl;
      for (int e = 0; e < list_len; ++e) {
        float sc = -__builtin_inff();
        long long rr = kNoRow;
        if (alive) src.get(q, li * list_len + e, sc, rr);
        const bool live = alive && rr >= 0 && rr != kNoRow && (R64 || rr != (long long)kEmptyRow);
        L.offer(sc, rr, live);
        alive = live && better64(sc, rr, L.ts, L.tr);
        if (!__any(alive)) break;
      }
    }
  } else {
    for (int64_t base = (int64_t)w * 64; base < n; base += (int64_t)P * NW * 64)
      merge_chunk<K, R64, P, NW>(src, q, base, n, lane, L);
  }
  if (lane < K) {
    ls_lds[w][lane] = L.ls;
    lr_lds[w][lane] = L.lr;
  }
  __syncthreads();
  rank_merge<K, NW>(ls_lds, lr_lds, ls_lds[NW], lr_lds[NW]);
  __syncthreads();
  if (tid < k_out) {
    const long long rr = lr_lds[NW][tid];
    const bool empty = rr == kNoRow;
    const float s = empty ? -__builtin_inff() : ls_lds[NW][tid];
    const long long r = empty ? -1 : rr + row_offset;
    if (out_rec) {
      out_rec[q * k_out + tid] = MergeRec{s, 0, r};
    } else {
      out_s[q * k_out + tid] = s;
      out_r[q * k_out + tid] = r;
    }
  }
}

// One index dtype's VALU launch (instantiated in valu_<dtype>.hip).
template <int DT>
int launch_valu_dt(const ValuPlan& p, const void* X, int nrows, int D, const void* Qf, int nq, float* cs, int* cr,
                   hipStream_t st, const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
  dim3 grid(p.blocks, p.q_slices);
  const size_t lds = (size_t)p.nqt * D * sizeof(float);
  const uint8_t* Xb = (const uint8_t*)X;
  if (p.nqt == 1)
    return launch_valu_k<DT, 1>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq, p.rows_per_wave, cs, cr,
                                p.n_lists, mask, tau, fo);
  if (p.nqt == 4)
    return launch_valu_k<DT, 4>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq, p.rows_per_wave, cs, cr,
                                p.n_lists, mask, tau, fo);
  if (p.nqt == 8)
    return launch_valu_k<DT, 8>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq, p.rows_per_wave, cs, cr,
                                p.n_lists, mask, tau, fo);
  return -1;
}
#define RFX_VALU_DT_DECL(NAME)                                                                           \
  int NAME(const ValuPlan& p, const void* X, int nrows, int D, const void* Qf, int nq, float* cs, int* cr,   \
           hipStream_t st, const uint32_t* mask, uint32_t* tau, const FusedOut& fo);
RFX_VALU_DT_DECL(launch_valu_f32)
RFX_VALU_DT_DECL(launch_valu_bf16)
RFX_VALU_DT_DECL(launch_valu_f16)
#undef RFX_VALU_DT_DECL

}  // namespace rfx
