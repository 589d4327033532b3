// k_scan_valu.hip — synthetic row generator, VALU fused scan + top-k, and top-k merge.
//
// Path: query×corpus inner-product scan + per-query top-k (the retrieval half of
// GeminiRag.ask_stream, backend/app/services/gemini_rag.py:517-551, which the reference runs
// remotely).  This file holds the small-batch (nq <= 8) scan; batched bf16/f16 queries go to
// the MFMA scan in k_scan_mfma.hip.
//
// Data layout in HBM: the vector store is row-major [rows][dim] of the index dtype, rows
// 16-B aligned (dim % 64 == 0).  A wave scans a contiguous row range; each 16-lane DPP row of
// the wave owns one corpus row per step (4 rows per wave-instruction, 256 contiguous bytes
// per row per load), so every load is a full-line coalesced dwordx4.
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {

// ---------------------------------------------------------------------------------------
// Synthetic rows: value(seed,row,col) = odd integer n in (-2^24, 2^24) from splitmix64; row
// normalised exactly (int64 sum of squares, f64 sqrt/div) then rounded to f32 then dtype.
// oracle/synth.py is the CPU restatement (bit-identical).
// ---------------------------------------------------------------------------------------

template <int DT>
__global__ __launch_bounds__(256) void synth_rows_kernel(uint64_t base, int64_t row0, int64_t n,
                                                         int dim, void* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nwaves) {
    const uint64_t rowkey = (uint64_t)(row0 + i) * (uint64_t)dim;
    long long ss = 0;
    for (int c = lane; c < dim; c += 64) {
      const long long v = synth_raw(base, rowkey + c);
      ss += v * v;
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) ss += __shfl_xor(ss, off);
    const double r = 1.0 / sqrt((double)ss);
    for (int c = lane; c < dim; c += 64) {
      const float x = (float)((double)synth_raw(base, rowkey + c) * r);
      if constexpr (DT == RFX_F32) {
        ((float*)out)[i * dim + c] = x;
      } else if constexpr (DT == RFX_BF16) {
        ((uint16_t*)out)[i * dim + c] = f32_to_bf16(x);
      } else {
        ((uint16_t*)out)[i * dim + c] = f32_to_f16(x);
      }
    }
  }
}

void launch_synth_rows(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, void* out,
                       hipStream_t st) {
  const uint64_t base = splitmix64(seed);
  const int64_t waves = n < 1 ? 1 : n;
  const int blocks = (int)std::min<int64_t>((waves + 3) / 4, 8192);
  if (dtype == RFX_F32)
    hipLaunchKernelGGL(synth_rows_kernel<RFX_F32>, dim3(blocks), dim3(256), 0, st, base, row0, n, dim, out);
  else if (dtype == RFX_BF16)
    hipLaunchKernelGGL(synth_rows_kernel<RFX_BF16>, dim3(blocks), dim3(256), 0, st, base, row0, n, dim, out);
  else
    hipLaunchKernelGGL(synth_rows_kernel<RFX_F16>, dim3(blocks), dim3(256), 0, st, base, row0, n, dim, out);
}

// Fill rows with quiet NaN (tombstone): NaN scores never pass the ranking rule.
__global__ void nan_rows_kernel(uint8_t* __restrict__ X, const int64_t* __restrict__ rows, int64_t n,
                                int64_t row_bytes, uint32_t pattern) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  uint8_t* p = X + rows[r] * row_bytes;
  for (int64_t b = threadIdx.x * 4; b < row_bytes; b += blockDim.x * 4) *(uint32_t*)(p + b) = pattern;
}

void launch_nan_rows(void* X, const int64_t* rows_d, int64_t n, int64_t row_bytes, int dtype,
                     hipStream_t st) {
  if (n <= 0) return;
  const uint32_t pattern = dtype == RFX_F32 ? 0x7fc00000u : (dtype == RFX_BF16 ? 0x7fc07fc0u : 0x7e007e00u);
  hipLaunchKernelGGL(nan_rows_kernel, dim3((unsigned)n), dim3(256), 0, st, (uint8_t*)X, rows_d, n,
                     row_bytes, pattern);
}

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
};

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

template <int DT, int NQT, int K, int VPL, bool FUSED>
__global__ __launch_bounds__(256) void scan_valu_kernel(const uint8_t* __restrict__ X, int nrows, int D,
                                                        const void* __restrict__ Qf, int nq,
                                                        int rows_per_wave, float* __restrict__ cand_s,
                                                        int* __restrict__ cand_r, int n_lists,
                                                        const uint32_t* __restrict__ mask,
                                                        uint32_t* __restrict__ tau, FusedOut fo) {
  constexpr int ESZ = DT == RFX_F32 ? 4 : 2;
  constexpr int EPV = 16 / ESZ;
  extern __shared__ __attribute__((aligned(16))) float q_lds[];  // [NQT][D]
  const int tid = threadIdx.x;
  const int lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int q0 = blockIdx.y * NQT;
  const int nqt = min(NQT, nq - q0);
  for (int i = tid; i < NQT * D; i += 256) {
    const int qi = i / D;
    const int64_t src = (int64_t)(q0 + qi) * D + (i - qi * D);
    q_lds[i] = qi >= nqt ? 0.f : FUSED ? query_elem<DT>(Qf, src) : ((const float*)Qf)[src];
  }
  __syncthreads();

  const int VPR = D * ESZ / 16;
  const int64_t RB = (int64_t)D * ESZ;
  const int wave_g = blockIdx.x * 4 + (tid >> 6);
  const int wb = (int)min((int64_t)wave_g * rows_per_wave, (int64_t)nrows);
  const int we = (int)min((int64_t)wb + rows_per_wave, (int64_t)nrows);

  WaveList<K> L[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) L[qi].init();

  float qr[NQT == 1 ? VPL * EPV : 1];
  if constexpr (NQT == 1) {
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int e = 0; e < EPV; ++e) {
        const int v = j + 16 * i;
        qr[i * EPV + e] = v < VPR ? q_lds[v * EPV + e] : 0.f;
      }
  }

  float cand[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) cand[qi] = 0.f;

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
  const int T = we > wb ? (we - wb + 63) / 64 * 16 : 0;  // iterations (16 per 64-row chunk)
  uint4 va[VPL], vb[VPL];
  if (T > 0) load_row(0, va);
  for (int t = 0; t < T; t += 2) {
    load_row(t + 1, vb);  // T is a multiple of 16: t + 1 < T
    score_row(t & 15, va);
    if (t + 2 < T) load_row(t + 2, va);
    score_row((t + 1) & 15, vb);
    if (((t + 2) & 15) == 0) {  // chunk done: offer its 64 rows
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
      if (lane == 0) bound = atomicMax(tau + q0 + qi, mine);
      bound = max((uint32_t)__builtin_amdgcn_readfirstlane(bound), mine);
    }
    if (lane < K) {
      const int64_t o = ((int64_t)(q0 + qi) * n_lists + blockIdx.x) * K + lane;
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
      last = old == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
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
      }
    } else {
      const AgentSrc src{cand_s, cand_r, n};
      for (int qi = 0; qi < nqt; ++qi) {
        merge_one<K, false, 4, true>(src, q0 + qi, K, fo.k_out, 0, fo.out_s, fo.out_r, nullptr);
        __syncthreads();
      }
    }
    if (tid < nqt && tau) tau[q0 + tid] = 0u;  // every block's bound updates precede its arrival
    if (tid == 0) fo.ctr[blockIdx.y] = 0u;
  }
}

// K values instantiated for the scan; runtime k is rounded up to one of these and only the
// first k entries of each list are used by the merge (lists are sorted).
#define RFX_VALU_K_LIST(X_) X_(4) X_(16) X_(64)

template <int DT, int NQT, int K>
static int launch_valu_vpl(int vpl, dim3 grid, size_t lds, hipStream_t st, const uint8_t* X, int nrows,
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
static int launch_valu_k(int kk, int vpl, dim3 grid, size_t lds, hipStream_t st, const uint8_t* X,
                         int nrows, int D, const void* Qf, int nq, int rpw, float* cs, int* cr,
                         int n_lists, const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
#define RFX_K(KV) \
  if (kk == KV) return launch_valu_vpl<DT, NQT, KV>(vpl, grid, lds, st, X, nrows, D, Qf, nq, rpw, cs, cr, n_lists, mask, tau, fo);
  RFX_VALU_K_LIST(RFX_K)
#undef RFX_K
  return -1;
}

int valu_k_slot(int k) { return k <= 4 ? 4 : (k <= 16 ? 16 : 64); }

ValuPlan plan_scan_valu(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  ValuPlan p{};
  const int esz = dtype == RFX_F32 ? 4 : 2;
  p.vpr = (int)((int64_t)D * esz / 16);
  p.vpl = (p.vpr + 15) / 16;
  p.k_slot = valu_k_slot(k);
  p.nqt = nq <= 1 ? 1 : (nq <= 4 ? 4 : 8);
  p.q_slices = (int)((nq + p.nqt - 1) / p.nqt);
  // Blocks: about kValuBlocks (one per CU), so that every CU streams the same share of the store — a
  // count just above a multiple of the CU count leaves most CUs idle for the last round (config 2
  // had 391 blocks on 256 CUs).  Rows per wave: a multiple of 4 (one row per 16-lane group and
  // iteration), at least 16.
  static const int blocks_env = [] {  // RFX_VALU_BLOCKS / RFX_VALU_RPW: ablation overrides
    const char* e = getenv("RFX_VALU_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  static const int rpw_env = [] {
    const char* e = getenv("RFX_VALU_RPW");
    return e ? atoi(e) : 0;
  }();
  const int64_t target_waves = 4 * (int64_t)(blocks_env > 0 ? blocks_env : kValuBlocks);
  int64_t rpw = (nrows + target_waves - 1) / target_waves;
  if (rpw < 16) rpw = 16;
  rpw = (rpw + 3) / 4 * 4;
  if (rpw_env >= 4) rpw = rpw_env / 4 * 4;
  int64_t waves = (nrows + rpw - 1) / rpw;
  if (waves < 1) waves = 1;
  p.rows_per_wave = (int)rpw;
  p.blocks = (int)((waves + 3) / 4);
  p.n_lists = p.blocks;  // one merged list per block
  p.ok = p.vpl <= 16 && p.k_slot <= 64 && (int64_t)D * esz % 16 == 0;
  return p;
}

static int launch_valu(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const void* Qf, int nq,
                       float* cs, int* cr, hipStream_t st, const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
  dim3 grid(p.blocks, p.q_slices);
  const size_t lds = (size_t)p.nqt * D * sizeof(float);
  const uint8_t* Xb = (const uint8_t*)X;
#define RFX_NQ(NQV)                                                                                \
  if (p.nqt == NQV) {                                                                              \
    if (dtype == RFX_F32)                                                                          \
      return launch_valu_k<RFX_F32, NQV>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq,       \
                                         p.rows_per_wave, cs, cr, p.n_lists, mask, tau, fo);                  \
    if (dtype == RFX_BF16)                                                                         \
      return launch_valu_k<RFX_BF16, NQV>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq,      \
                                          p.rows_per_wave, cs, cr, p.n_lists, mask, tau, fo);                 \
    return launch_valu_k<RFX_F16, NQV>(p.k_slot, p.vpl, grid, lds, st, Xb, nrows, D, Qf, nq,         \
                                       p.rows_per_wave, cs, cr, p.n_lists, mask, tau, fo);                    \
  }
  RFX_NQ(1) RFX_NQ(4) RFX_NQ(8)
#undef RFX_NQ
  return -1;
}

int launch_scan_valu(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const float* Qf, int nq,
                     float* cs, int* cr, hipStream_t st, const uint32_t* mask, uint32_t* tau) {
  return launch_valu(p, X, nrows, D, dtype, Qf, nq, cs, cr, st, mask, tau, FusedOut{nullptr, 0, nullptr, nullptr});
}

int launch_search_valu_fused(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const void* Q, int nq,
                             float* cs, int* cr, uint32_t* state, int k, float* out_s, int64_t* out_r,
                             hipStream_t st, const uint32_t* mask) {
  // state: [kFusedMaxNq] bounds then [q_slices] counters, all zero (and left zero)
  return launch_valu(p, X, nrows, D, dtype, Q, nq, cs, cr, st, mask, state,
                     FusedOut{state + kValuFusedMaxNq, k, out_s, out_r});
}

// Diagnostic streaming read (HBM ceiling calibration): every byte read once with dwordx4.
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

void launch_stream_read(const void* p, int64_t bytes, uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(256 * 16), dim3(256), 0, st, (const uint4*)p, bytes / 16, out);
}

// Widen index-dtype queries to f32 (exact).
__global__ void widen_queries_kernel(const void* __restrict__ Q, int64_t n, int dtype, float* __restrict__ out,
                                     uint32_t* __restrict__ tau, int64_t n_tau) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_tau; i += (int64_t)gridDim.x * blockDim.x)
    tau[i] = 0u;  // the scan's per-query pruning bounds start empty
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (dtype == RFX_F32)
      out[i] = ((const float*)Q)[i];
    else if (dtype == RFX_BF16)
      out[i] = bf16_to_f32(((const uint16_t*)Q)[i]);
    else
      out[i] = f16_to_f32(((const uint16_t*)Q)[i]);
  }
}

void launch_widen_queries(const void* Q, int64_t n, int dtype, float* out, hipStream_t st, uint32_t* tau,
                          int64_t n_tau) {
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(widen_queries_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(256), 0, st, Q, n, dtype, out, tau,
                     tau ? n_tau : 0);
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

template <int K, bool R64, bool SORTED, class Src>
__global__ __launch_bounds__(512) void merge_kernel(Src src, int list_len, int k_out, int64_t row_offset,
                                                    float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                                    MergeRec* __restrict__ out_rec) {
  merge_one<K, R64, 8, SORTED>(src, (int64_t)blockIdx.x, list_len, k_out, row_offset, out_s, out_r, out_rec);
}

int launch_topk_merge_lists(const float* cs, const void* cr, int rows_are_i64, int64_t nq, int64_t n_cand,
                            int list_len, int k, int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec,
                            hipStream_t st, bool sorted) {
  const int kk = valu_k_slot(k);
  if (nq <= 0) return 0;
  if (list_len < 1 || (list_len > 1 && n_cand % list_len != 0)) {
    list_len = 1;
    sorted = false;
  }
  MergeRec* rec = (MergeRec*)out_rec;
#define RFX_M2(KV, R, S)                                                                                  \
  hipLaunchKernelGGL((merge_kernel<KV, R, S, FlatSrc<R>>), dim3((unsigned)nq), dim3(512), 0, st,          \
                     FlatSrc<R>{cs, cr, n_cand}, list_len, k, row_offset, out_s, out_r, rec)
#define RFX_M(KV)                                                                                     \
  if (kk == KV) {                                                                                     \
    if (rows_are_i64 && sorted)                                                                       \
      RFX_M2(KV, true, true);                                                                         \
    else if (rows_are_i64)                                                                            \
      RFX_M2(KV, true, false);                                                                        \
    else if (sorted)                                                                                  \
      RFX_M2(KV, false, true);                                                                        \
    else                                                                                              \
      RFX_M2(KV, false, false);                                                                       \
    return 0;                                                                                         \
  }
  RFX_VALU_K_LIST(RFX_M)
#undef RFX_M
#undef RFX_M2
  return -1;
}

int launch_topk_merge(const float* cs, const void* cr, int rows_are_i64, int64_t nq, int64_t n_cand, int k,
                      int64_t row_offset, float* out_s, int64_t* out_r, hipStream_t st) {
  return launch_topk_merge_lists(cs, cr, rows_are_i64, nq, n_cand, 1, k, row_offset, out_s, out_r, nullptr, st);
}

int launch_merge_gathered(const void* rec, int world, int64_t nq, int k, float* out_s, int64_t* out_r,
                          hipStream_t st) {
  const int kk = valu_k_slot(k);
  if (nq <= 0) return 0;
  GatheredSrc src{(const MergeRec*)rec, nq, k, (int64_t)world * k};
#define RFX_M(KV)                                                                                     \
  if (kk == KV) {                                                                                     \
    hipLaunchKernelGGL((merge_kernel<KV, true, true, GatheredSrc>), dim3((unsigned)nq), dim3(512), 0, st, \
                       src, k, k, 0, out_s, out_r, nullptr);                                          \
    return 0;                                                                                         \
  }
  RFX_VALU_K_LIST(RFX_M)
#undef RFX_M
  return -1;
}

}  // namespace rfx
