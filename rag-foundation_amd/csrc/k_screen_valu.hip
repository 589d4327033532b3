// k_screen_valu.hip — kernel 11: the exact two-pass scan for a lone question or a handful (nq <= 8;
// BASELINE config 2: 100k × 768 f32, nq 1, k 10, and the adapter's un-batched questions), in ONE
// launch: int8 screen of the index's int8 copy on v_dot4_i32_i8, exact re-score of the rows that can
// still reach the top-k, the final merge in the last block.  A gated launch of the exact one-launch
// VALU search (k_scan_valu.h) follows and runs only when the screen cannot prove its answer.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// The int8 copy and the exactness argument are kernel 10's (k_scan_screen.h): per
// 32-row tile scale s_t, per query s_y and e2 = 2 E_q / s_y (rounded up), screen score A = s_t D.
// With LB <= a_K (the K-th best A over live rows, K >= k) every row of the exact top-k has
// A >= LB - e2.  Here:
//   * each wave keeps the K best A of its rows per query (WaveList) and dmax, the best A it had to
//     drop (rejected or evicted); the block merges its 4 wave lists (dropping into dmax too);
//   * each wave publishes its list after its first 64 rows, and the block its merged list at the
//     end, to the query's 16 bound slots (row r to slot r % 16, agent atomic max): a slot holds the
//     A of one live row and different slots hold different rows, so the k-th largest slot, LB, is a
//     lower bound of a_k — and close to it once every wave's first rows are in;
//   * the block re-scores exactly (f64 sum of exact products, rounded to f32) every list entry with
//     A >= max(k-th slot read, own K-th) - e2 <= LB - e2, so the entries it skips cannot be in the top-k;
//   * the last block merges the exact scores.  When some dmax reaches LB - e2 a dropped row might
//     have belonged to the top-k: it sets the gate and the exact search rewrites the answer.
// Algorithmic bytes: N·d codes + ⌈N/32⌉·16 tile records + the re-scored rows (a few per query).
#include "k_scan_valu.h"

namespace rfx {
namespace {

constexpr int kK = 16;  // A-list length (k <= 16)

template <int DT>
__device__ __forceinline__ float qelem(const void* Q, int64_t i) {
  if constexpr (DT == RFX_F32)
    return ((const float*)Q)[i];
  else if constexpr (DT == RFX_BF16)
    return bf16_to_f32(((const uint16_t*)Q)[i]);
  else
    return f16_to_f32(((const uint16_t*)Q)[i]);
}

__device__ __forceinline__ float f32_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_inff());
  return f;
}

__device__ __forceinline__ float unord_f32(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// the k-th largest of a query's 16 bound slots (orderable A; 0 = empty), k <= 16: bitonic sort
__device__ __forceinline__ uint32_t slots_kth(const uint32_t* sl, int k, bool agent) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    v[i] = agent ? __hip_atomic_load(sl + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : sl[i];
#pragma unroll
  for (int kk = 2; kk <= 16; kk <<= 1)
#pragma unroll
    for (int jj = kk >> 1; jj > 0; jj >>= 1)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int l = i ^ jj;
        if (l > i) {
          const uint32_t a = v[i], b = v[l];
          const bool desc = (i & kk) == 0;
          v[i] = desc ? max(a, b) : min(a, b);
          v[l] = desc ? min(a, b) : max(a, b);
        }
      }
  uint32_t r = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) r = i == k - 1 ? v[i] : r;
  return r;
}

// D / 16 bytes of int8 codes per lane of a 16-lane row group: chunk c = j + 16 i (16 B each)
template <int D>
struct Codes {
  static constexpr int C = D / 256;  // 16-B chunks per lane (3 at d 768, 4 at d 1024)
  uint4 v[C];
};

template <int DT, int D, int NQT>
__global__ __launch_bounds__(256) void screen_valu_kernel(const int8_t* __restrict__ X8, const uint4* __restrict__ tmeta,
                                                          const uint32_t* __restrict__ stats, int nrows,
                                                          const void* __restrict__ X, const void* __restrict__ Q, int nq,
                                                          int rows_per_wave, const uint32_t* __restrict__ mask,
                                                          uint32_t* __restrict__ state, float* __restrict__ cand_s,
                                                          int* __restrict__ cand_r, int k_out, float* __restrict__ out_s,
                                                          int64_t* __restrict__ out_r, int force) {
  constexpr int C = D / 256;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int n_lists = gridDim.x;
  // state (per index and stream, zero on entry and left zero): [0] arrival counter, [16..24) the
  // queries' dmax, [24] the fallback gate (written, not reset), [32 + 16 q ..) query q's bound slots
  uint32_t* const ctr = state;
  uint32_t* const dmx = state + 16;
  uint32_t* const gate = state + 24;
  uint32_t* const slots = state + 32;

  // ---- 1. query codes and e2 (every block, identically): wave w quantises queries w, w + 4 ------
  __shared__ __attribute__((aligned(16))) int8_t qc_lds[NQT][D];
  __shared__ float e2_lds[NQT];
  {
    const double xm = (double)__uint_as_float(stats[0]), em = (double)__uint_as_float(stats[1]);
    for (int qi = w; qi < NQT; qi += 4) {
      constexpr int PL = D / 64;  // elements per lane
      float y[PL];
      float am = 0.f;
#pragma unroll
      for (int e = 0; e < PL; ++e) {
        y[e] = qi < nq ? qelem<DT>(Q, (int64_t)qi * D + lane + 64 * e) : 0.f;
        am = fmaxf(am, fabsf(y[e]));
      }
#pragma unroll
      for (int off = 32; off; off >>= 1) am = fmaxf(am, __shfl_xor(am, off));
      const float s = am > 0.f ? __fdiv_rn(am, 127.f) : 0.f;
      double ey = 0.0;
      long long cc = 0;
#pragma unroll
      for (int e = 0; e < PL; ++e) {
        int c = 0;
        if (s > 0.f) c = (int)fminf(fmaxf(rintf(__fdiv_rn(y[e], s)), -127.f), 127.f);
        qc_lds[qi][lane + 64 * e] = (int8_t)c;
        const double dd = (double)y[e] - (double)s * (double)c;
        ey += dd * dd;
        cc += (long long)c * c;
      }
#pragma unroll
      for (int off = 32; off; off >>= 1) {
        ey += __shfl_xor(ey, off);
        cc += __shfl_xor(cc, off);
      }
      if (lane == 0) {
        float e2 = 0.f;
        if (s > 0.f) {
          const double yh = (double)s * sqrt((double)cc);
          const double eq = xm * sqrt(ey) + em * yh;
          e2 = f32_up((2.0 * eq + 4e-7 * (xm + em) * yh) * (1.0 + 1e-5) / (double)s);
        }
        e2_lds[qi] = e2;
      }
    }
  }
  __syncthreads();
  Codes<D> qv[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi)
#pragma unroll
    for (int i = 0; i < C; ++i) qv[qi].v[i] = *(const uint4*)(&qc_lds[qi][16 * (j + 16 * i)]);

  // ---- 2. the int8 row stream: iteration t scores rows wb + 64 (t >> 4) + 4 (t & 15) + g ----------
  const int wave_g = blockIdx.x * 4 + w;
  const int wb = (int)min((int64_t)wave_g * rows_per_wave, (int64_t)nrows);
  const int we = (int)min((int64_t)wb + rows_per_wave, (int64_t)nrows);
  const int T = we > wb ? (we - wb + 15) / 16 * 4 : 0;
  WaveList<kK> L[NQT];
  float dm[NQT];  // per lane: the best A this wave dropped (rejected at offer time or evicted)
  float cand[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) {
    L[qi].init();
    dm[qi] = -__builtin_inff();
    cand[qi] = __builtin_nanf("");
  }
  auto load_row = [&](int t, Codes<D>& v) {
    const int row = wb + 64 * (t >> 4) + 4 * (t & 15) + g;
    const int8_t* rp = X8 + (int64_t)(row < we ? row : wb) * D;
#pragma unroll
    for (int i = 0; i < C; ++i) v.v[i] = *(const uint4*)(rp + 16 * (j + 16 * i));
  };
  auto score_row = [&](int t, const Codes<D>& v) {
    const int row = wb + 64 * (t >> 4) + 4 * (t & 15) + g;
    const uint4 md = tmeta[(row < we ? row : wb) >> 5];  // the tile's {scale, live word}: cache hits
    const float st = __uint_as_float(md.x);
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      int acc = 0;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        acc = __builtin_amdgcn_sdot4((int)v.v[i].x, (int)qv[qi].v[i].x, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].y, (int)qv[qi].v[i].y, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].z, (int)qv[qi].v[i].z, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].w, (int)qv[qi].v[i].w, acc, false);
      }
      const float dsum = row16_sum((float)acc);  // |partial sums| < 2^24: exact in f32
      const float a = dsum * st;                 // A = s_t D, one rounding (as kernel 10)
      const bool live = row < we && ((md.y >> (row & 31)) & 1u) && (mask == nullptr || row_allowed(mask, row));
      if (j == (t & 15)) cand[qi] = live ? a : __builtin_nanf("");
    }
  };
  auto offer = [&](int qi, float a, int row) {
    // offer one candidate per lane; record in dm what the list does not keep
    WaveList<kK>& l = L[qi];
    const bool valid = a == a;  // NaN = dead / masked / past the end
    if (valid && !better(a, row, l.ts, l.tr)) dm[qi] = fmaxf(dm[qi], a);
    uint64_t m = __ballot(valid && better(a, row, l.ts, l.tr));
    while (m) {
      const int src = __builtin_ctzll(m);
      m &= m - 1;
      const float s = readlane_f(a, src);
      const int r = readlane_i(row, src);
      if (!better(s, r, l.ts, l.tr)) {  // the threshold rose meanwhile: dropped
        if (lane == src) dm[qi] = fmaxf(dm[qi], s);
        continue;
      }
      const float ev = readlane_f(l.ls, kK - 1);  // evicted (-inf while the list is not full)
      if (lane == 0) dm[qi] = fmaxf(dm[qi], ev);
      const bool b = (lane < kK) && better(l.ls, l.lr, s, r);
      const int pos = __popcll(__ballot(b));
      const float us = lane_shr1(l.ls);
      const int ur = lane_shr1(l.lr);
      if (lane > pos && lane < kK) {
        l.ls = us;
        l.lr = ur;
      }
      if (lane == pos) {
        l.ls = s;
        l.lr = r;
      }
      l.ts = readlane_f(l.ls, kK - 1);
      l.tr = readlane_i(l.lr, kK - 1);
    }
  };
  Codes<D> va, vb, vc, vd;
  if (T > 0) {
    load_row(0, va);
    load_row(1, vb);
    load_row(2, vc);
  }
  for (int t = 0; t < T; t += 4) {
    load_row(t + 3, vd);
    score_row(t, va);
    load_row(t + 4, va);
    score_row(t + 1, vb);
    load_row(t + 5, vb);
    score_row(t + 2, vc);
    load_row(t + 6, vc);
    score_row(t + 3, vd);
    if (((t + 4) & 15) == 0 || t + 4 >= T) {  // a 64-row chunk scored: every lane holds one row
      const int crow = wb + 64 * (t >> 4) + j * 4 + g;
#pragma unroll
      for (int qi = 0; qi < NQT; ++qi) {
        offer(qi, crow < we ? cand[qi] : __builtin_nanf(""), crow);
        cand[qi] = __builtin_nanf("");
        // the first chunk's list goes to the bound slots at once: the blocks run in step, so a bound
        // published only at the end would reach no block in time to prune its re-scoring
        if (t < 16 && qi < nq && lane < kK && L[qi].lr != kEmptyRow)
          __hip_atomic_fetch_max(slots + 16 * qi + (L[qi].lr & 15), ord_f32(L[qi].ls), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  // ---- 3. block list per query, its K-th A published, bound read --------------------------------
  __shared__ float ms[4][NQT][kK];
  __shared__ int mr[4][NQT][kK];
  __shared__ float wdm[4][NQT];
  uint32_t seen[(NQT + 3) / 4];  // the k-th slot as it stands now (any value read is a valid bound)
#pragma unroll
  for (int u = 0; u < (NQT + 3) / 4; ++u) {
    const int qi = w + 4 * u;
    seen[u] = qi < nq ? slots_kth(slots + 16 * qi, k_out, true) : 0u;
  }
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) {
    if (lane < kK) {
      ms[w][qi][lane] = L[qi].ls;
      mr[w][qi][lane] = L[qi].lr;
    }
    float d = dm[qi];
#pragma unroll
    for (int off = 32; off; off >>= 1) d = fmaxf(d, __shfl_xor(d, off));
    if (lane == 0) wdm[w][qi] = d;
  }
  __syncthreads();
  __shared__ float bA[NQT][kK];
  __shared__ int bR[NQT][kK];
  __shared__ float bCut[NQT];
  for (int qi = w; qi < NQT; qi += 4) {
    WaveList<kK> M;
    M.init();
#pragma unroll
    for (int src = 0; src < 4; ++src) {
      const bool v = lane < kK && mr[src][qi][lane] != kEmptyRow;
      M.offer(v ? ms[src][qi][lane] : -__builtin_inff(), v ? mr[src][qi][lane] : kEmptyRow, v);
    }
    // entries of the wave lists the block list does not hold: strictly worse than its K-th entry
    float d = fmaxf(fmaxf(wdm[0][qi], wdm[1][qi]), fmaxf(wdm[2][qi], wdm[3][qi]));
#pragma unroll
    for (int src = 0; src < 4; ++src) {
      const bool v = lane < kK && mr[src][qi][lane] != kEmptyRow;
      const float s = v ? ms[src][qi][lane] : -__builtin_inff();
      if (v && better(M.ts, M.tr, s, mr[src][qi][lane])) d = fmaxf(d, s);
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) d = fmaxf(d, __shfl_xor(d, off));
    const float kth = readlane_f(M.ls, kK - 1);
    const bool full = readlane_i(M.lr, kK - 1) != kEmptyRow;
    if (qi < nq) {
      if (lane < kK && M.lr != kEmptyRow)
        __hip_atomic_fetch_max(slots + 16 * qi + (M.lr & 15), ord_f32(M.ls), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0 && d > -__builtin_inff())
        __hip_atomic_fetch_max(dmx + qi, ord_f32(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t sn = seen[(qi - w) / 4];
    float b = sn ? unord_f32(sn) : -__builtin_inff();
    if (full) b = fmaxf(b, kth);
    if (lane < kK) {
      bA[qi][lane] = M.ls;
      bR[qi][lane] = M.lr;
    }
    if (lane == 0) bCut[qi] = b > -__builtin_inff() ? b - e2_lds[qi] : -__builtin_inff();
  }
  __syncthreads();

  // ---- 4. exact re-score of the block's entries at or above its cut: 16 lanes per entry, 16 entries
  // at a time, every row's loads in flight together (one memory latency per round) ---------------
  {
    constexpr int ESZ = DT == RFX_F32 ? 4 : 2;
    constexpr int EPV = 16 / ESZ;         // elements per 16-B load
    constexpr int VPL = D * ESZ / 256;    // 16-B loads per lane (a 16-lane group covers the row)
    const int grp = tid >> 4, gl = tid & 15;
    for (int e0 = 0; e0 < NQT * kK; e0 += 16) {
      const int e = e0 + grp, qi = e / kK, i = e - qi * kK;
      const int r = bR[qi][i];
      const bool go = qi < nq && r != kEmptyRow && bA[qi][i] >= bCut[qi];
      double acc = 0.0;
      if (go) {
        uint4 xv[VPL], yv[VPL];
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
          xv[u] = *(const uint4*)((const uint8_t*)X + (int64_t)r * D * ESZ + (int64_t)(gl + 16 * u) * 16);
          yv[u] = *(const uint4*)((const uint8_t*)Q + (int64_t)qi * D * ESZ + (int64_t)(gl + 16 * u) * 16);
        }
#pragma unroll
        for (int u = 0; u < VPL; ++u)
#pragma unroll
          for (int ee = 0; ee < EPV; ++ee) acc += (double)elem<DT>(xv[u], ee) * (double)elem<DT>(yv[u], ee);
      }
#pragma unroll
      for (int off = 8; off; off >>= 1) acc += __shfl_xor(acc, off);  // within the 16-lane group
      if (gl == 0 && qi < nq) {
        const int64_t o = ((int64_t)qi * n_lists + blockIdx.x) * kK + i;
        __hip_atomic_store((uint32_t*)cand_s + o, __float_as_uint(go ? (float)acc : -__builtin_inff()),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cand_r + o, go ? r : kEmptyRow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  // ---- 5. the last block: check the drops against LB - e2, merge the exact scores ---------------
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __shared__ int fail;
  if (tid == 0) fail = force;
  __syncthreads();
  if (tid < nq) {
    const uint32_t lb = slots_kth(slots + 16 * tid, k_out, true);
    const uint32_t d = __hip_atomic_load(dmx + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // no bound (fewer than k slots filled) with drops, or a drop at or above LB - e2: not proven
    if (d && (!lb || unord_f32(d) >= unord_f32(lb) - e2_lds[tid])) atomicOr(&fail, 1);
  }
  __syncthreads();
  if (!fail) {
    const int64_t n = (int64_t)n_lists * kK;
    __shared__ float bs[kFusedLdsCand];
    __shared__ int br[kFusedLdsCand];
    for (int qi = 0; qi < nq; ++qi) {
      const int64_t qo = (int64_t)qi * n;
      if (n <= kFusedLdsCand) {
        for (int i = tid; i < (int)n; i += 256) {
          bs[i] = __uint_as_float(__hip_atomic_load((const uint32_t*)cand_s + qo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          br[i] = __hip_atomic_load(cand_r + qo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        merge_one<kK, false, 4, false>(LdsSrc{bs, br, n}, qi, kK, k_out, 0, out_s, out_r, nullptr);
      } else {
        merge_one<kK, false, 4, false>(AgentSrc{cand_s, cand_r, n}, qi, kK, k_out, 0, out_s, out_r, nullptr);
      }
      __syncthreads();
    }
  }
  if (tid < 8) dmx[tid] = 0u;
  if (tid < 8 * 16) slots[tid] = 0u;
  if (tid == 0) {
    *gate = fail ? 1u : 0u;  // read by the gated exact search that follows on the stream
    *ctr = 0u;
  }
}

}  // namespace

// One launch: grid (blocks) × 256 threads, one query slice of up to 8 queries.
int launch_screen_valu(const ValuPlan& p, const int8_t* X8, const void* tmeta, const uint32_t* stats, int nrows, int D,
                       int dtype, const void* X, const void* Q, int nq, const uint32_t* mask, uint32_t* state,
                       float* cs, int* cr, int k, float* out_s, int64_t* out_r, int force, hipStream_t st) {
  if (nq < 1 || nq > 8 || k < 1 || k > kK || (D != 768 && D != 1024)) return -1;
  if ((int64_t)p.blocks * kK > (int64_t)1 << 30) return -1;
  const dim3 grid((unsigned)p.blocks);
#define RFX_SV(DTV, DV, NQ)                                                                                      \
  hipLaunchKernelGGL((screen_valu_kernel<DTV, DV, NQ>), grid, dim3(256), 0, st, X8, (const uint4*)tmeta, stats, nrows, \
                     X, Q, nq, p.rows_per_wave, mask, state, cs, cr, k, out_s, out_r, force)
#define RFX_SV_D(DTV)                  \
  if (D == 768) {                      \
    if (nq == 1)                       \
      RFX_SV(DTV, 768, 1);             \
    else                               \
      RFX_SV(DTV, 768, 8);             \
  } else {                             \
    if (nq == 1)                       \
      RFX_SV(DTV, 1024, 1);            \
    else                               \
      RFX_SV(DTV, 1024, 8);            \
  }
  if (dtype == RFX_F32) {
    RFX_SV_D(RFX_F32)
  } else if (dtype == RFX_BF16) {
    RFX_SV_D(RFX_BF16)
  } else {
    RFX_SV_D(RFX_F16)
  }
#undef RFX_SV_D
#undef RFX_SV
  return 0;
}

}  // namespace rfx
