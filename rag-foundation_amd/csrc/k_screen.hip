// k_screen.hip — the exact two-pass scan around kernel 10 (k_scan_screen.h): the int8 copy of the
// store (per-tile quantiser), the per-batch query quantiser, and the select kernel that finds each
// query's survivors, re-scores them exactly from the stored rows and writes the top-k.  DESIGN §4.10.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551);
// the store write of upload_file (gemini_rag.py:307-352) keeps the int8 copy current.
// oracle/screen.py restates every step; the codes, tile scales and live words are bit-exact with it
// (one correctly rounded IEEE op per float step: __fdiv_rn, rintf).
#include "k_scan_screen.h"
#ifdef RFX_DEBUG_BUILD
namespace rfx {
namespace {
// debug library only: per block (query < 256) the 100-MHz wall clock at the select's phase ends
// (tools/select_phases.py via rfx_dbg_select_times)
__device__ unsigned long long g_sel_t[256][8];
}  // namespace
}  // namespace rfx
#define RFX_SEL_T(i) \
  if (threadIdx.x == 0 && blockIdx.x < 256) ::rfx::g_sel_t[blockIdx.x][i] = wall_clock64();
#endif
#include "k_select.h"

namespace rfx {
namespace k10 {
#define RFX_K10_DECL(NAME)                                                                                    \
  int NAME(int kl, dim3 grid, hipStream_t st, const int8_t* X, const uint4* tm, const uint32_t* sts,           \
           const int8_t* Qc, const float* qe2, int nq, int ntiles, uint32_t* tau, float* cs, int* cr,          \
           uint32_t* dr, int64_t n_lists, const uint32_t* mask, uint32_t* xb, uint32_t* xw);
RFX_K10_DECL(launch_768)
RFX_K10_DECL(launch_1024)
RFX_K10_DECL(launch_768_w2)
RFX_K10_DECL(launch_1024_w2)
}  // namespace k10
namespace k10q {
RFX_K10_DECL(launch_768)
}  // namespace k10q
#undef RFX_K10_DECL

namespace {

using mfc::ord;
using mfc::unord;

template <int DT>
__device__ __forceinline__ float widen(uint16_t h) {
  if constexpr (DT == RFX_BF16)
    return __uint_as_float((uint32_t)h << 16);
  else
    return f16_to_f32(h);
}

// f64 -> f32 rounded up (an upper bound stays an upper bound)
__device__ __forceinline__ float f32_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_inff());
  return f;
}

__device__ __forceinline__ int8_t code_of(float x, float s) {
  const float c = rintf(__fdiv_rn(x, s));
  return (int8_t)fminf(fmaxf(c, -127.f), 127.f);
}

// ---- the int8 copy: one 256-thread block per 32-row tile ----------------------------------------
// Per tile a 16-B record {f32 scale, u32 live word (bit r = row r live), 0, 0}.
// thread t: row t >> 3, segment t & 7 (D / 8 elements).  A row is dead (tombstone, NaN tail) when any
// element is NaN: code 0, live bit clear, excluded from the scale.  s_t = amax / 127 over the live
// rows (0 for a tile without any), c = clamp(rint(x / s_t), ±127).  stats[0] / stats[1] grow to the
// max over live rows of ||x|| and ||x − s_t c|| (f64 sums, rounded up to f32, atomicMax on the bits),
// stats[2] to the max tile scale.
// 8 consecutive stored elements from element index i (16-B aligned groups), widened exactly
template <int DT>
__device__ __forceinline__ void load8(const void* X, int64_t i, float (&f)[8]) {
  if constexpr (DT == RFX_F32) {
    const uint4 a = *(const uint4*)((const float*)X + i), b = *(const uint4*)((const float*)X + i + 4);
    const uint32_t u[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = __uint_as_float(u[e]);
  } else {
    const uint4 v = *(const uint4*)((const uint16_t*)X + i);
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = widen<DT>((uint16_t)(e & 1 ? u[e >> 1] >> 16 : u[e >> 1] & 0xffffu));
  }
}

template <int DT, int D>
__global__ __launch_bounds__(256) void screen_quantize_kernel(const void* __restrict__ X, int64_t tile0,
                                                              const int64_t* __restrict__ tiles,
                                                              int8_t* __restrict__ codes, uint4* __restrict__ tmeta,
                                                              uint32_t* __restrict__ stats) {
  constexpr int PER = D / 8;
  const int64_t tile = tiles ? tiles[blockIdx.x] : tile0 + blockIdx.x;
  const int t = threadIdx.x, row = t >> 3, seg = t & 7;
  const int64_t r = tile * 32 + row;
  const int64_t xr = r * D + seg * PER;  // element index of the thread's segment
  __shared__ float wmax[4];
  __shared__ uint32_t word;
  if (t == 0) word = 0u;
  bool nan = false;
  float am = 0.f;
#pragma unroll 4
  for (int i = 0; i < PER; i += 8) {
    float fv[8];
    load8<DT>(X, xr + i, fv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = fv[e];
      nan |= f != f;
      am = fmaxf(am, fabsf(f));
    }
  }
  // the 8 threads of a row are 8 consecutive lanes of one wave
  int dead = nan;
  dead |= __shfl_xor(dead, 1);
  dead |= __shfl_xor(dead, 2);
  dead |= __shfl_xor(dead, 4);
  float m = dead ? 0.f : am;
#pragma unroll
  for (int off = 32; off; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((t & 63) == 0) wmax[t >> 6] = m;
  __syncthreads();
  const float amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  const float s = amax > 0.f ? __fdiv_rn(amax, 127.f) : 0.f;
  double xx = 0.0, ee = 0.0;
  int8_t* cw = codes + r * D + seg * PER;
#pragma unroll 4
  for (int i = 0; i < PER; i += 8) {
    float fv[8];
    load8<DT>(X, xr + i, fv);
    uint32_t pk[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = fv[e];
      const int8_t c = (!dead && s > 0.f) ? code_of(f, s) : (int8_t)0;
      pk[e >> 2] |= (uint32_t)(uint8_t)c << (8 * (e & 3));
      if (!dead) {
        const double d = (double)f - (double)s * (double)c;  // exact: both terms fit 53 bits
        xx += (double)f * (double)f;
        ee += d * d;
      }
    }
    *(uint2*)(cw + i) = uint2{pk[0], pk[1]};
  }
  xx += __shfl_xor(xx, 1);
  xx += __shfl_xor(xx, 2);
  xx += __shfl_xor(xx, 4);
  ee += __shfl_xor(ee, 1);
  ee += __shfl_xor(ee, 2);
  ee += __shfl_xor(ee, 4);
  if (seg == 0 && !dead) {
    atomicMax(stats + 0, __float_as_uint(f32_up(sqrt(xx))));  // non-negative floats order as u32
    atomicMax(stats + 1, __float_as_uint(f32_up(sqrt(ee))));
    atomicOr(&word, 1u << row);
  }
  __syncthreads();
  if (t == 0) {
    tmeta[tile] = uint4{__float_as_uint(s), word, 0u, 0u};  // kernel 10 DMAs this record per tile
    atomicMax(stats + 2, __float_as_uint(s));              // the max tile scale (its fast-path bound)
  }
}

// ---- per batch: query codes and e2 (one wave per query) -------------------------------------------
// s_y = amax / 127, c = clamp(rint(y / s_y)); E_q = Xmax ||y − s_y c|| + Emax ||s_y c|| (Cauchy-Schwarz,
// k_scan_screen.h); e2 = (2 E_q + 4e-7 (Xmax + Emax) ||s_y c|| + 2.4e-7 Xmax (||s_y c|| + ||y - s_y c||))
// (1 + 1e-5) / s_y rounded up: the 4e-7 term covers the f32 roundings of A = s_t D (2^-24 relative,
// twice) and of the bound subtraction, the 2.4e-7 term two f32 ulps of the k-th exact score (>= 2^-23
// |score|, |score| <= Xmax ||y||): under the score rule (fl32 of the exact dot desc, row asc) a row
// whose exact score is below the k-th but rounds to the same f32 and has a smaller row id belongs to
// the answer, so it must survive; the 1e-5 the f64 norms.  Also zeroes the query's threshold slots and (block 0) the
// fallback gate.  Padded queries (q >= nq) get code 0 and e2 0.
// Kernel 10's XCD table, one per device (k_scan_screen.h: the tile split across the 8 XCDs): [0, 8)
// weights (1024 = 1.0, 0 = not measured yet), [8, 16) the blocks' durations (10-ns ticks) and [16, 24)
// their tiles per XCD, summed by kernel 10 since the last query quantiser.
__device__ uint32_t g_xcd_w[24];

// The seed (round 6): kernel 10's blocks start with no bound, so their first tiles pass nearly every value
// (16 slow-path trips per wave at tiles 0 and 1: a third of all trips at the 8-GPU shard).  The
// quantiser gives each query a bound to start from: the KL-th best screen score A = fl(D s_t) over kSeedRows
// live, allowed sample rows spread over the store (rows i * rows / S).  They are distinct live rows, so the
// KL-th best of their A is at most the KL-th best over all live rows, hence at most a_k (KL >= k): a valid
// lower bound, like the slot table's.  No seed (0) with fewer than KL such rows.
constexpr int kSeedRows = 256;

template <int DT, int D>
__global__ __launch_bounds__(256) void screen_queries_kernel(const void* __restrict__ Q, int nq, int nq_pad,
                                                             int8_t* __restrict__ Qc, float* __restrict__ qe2,
                                                             const uint32_t* __restrict__ stats,
                                                             uint32_t* __restrict__ tau, uint32_t* __restrict__ gate,
                                                             uint32_t* __restrict__ ftau, int ftau_nq,
                                                             uint32_t* __restrict__ xb, const int8_t* __restrict__ X8,
                                                             const uint4* __restrict__ tmeta, int nrows,
                                                             const uint32_t* __restrict__ mask, int kl,
                                                             uint32_t* __restrict__ seed) {
  constexpr int NM = D / 256;
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) *gate = 0u;
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    // Kernel 10's split for this launch (lanes 0..7 = XCDs): the speed each XCD measured since the last
    // quantiser (tiles per tick, the sums taken and reset), its weight moved half-way to its share of
    // the mean speed (clamped to [0.5, 2]); the snapshot in the workspace is what every block of this
    // launch reads.  Concurrent launches on other streams only blur the measurement.
    const int x = threadIdx.x;
    uint32_t d = 0u, n = 0u, w = 1024u;
    if (x < 8) {
      d = __hip_atomic_exchange(&g_xcd_w[8 + x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      n = __hip_atomic_exchange(&g_xcd_w[16 + x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w = __hip_atomic_load(&g_xcd_w[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w = w == 0u ? 1024u : w < 512u ? 512u : w > 2048u ? 2048u : w;
    }
    const float sp = d && n ? (float)n / (float)d : 0.f;
    float sum = sp;
    int have = x < 8 && sp > 0.f ? 1 : 0;
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      sum += __shfl_xor(sum, off);
      have += __shfl_xor(have, off);
    }
    if (x < 8) {
      if (have == 8 && sum > 0.f) {
        const float want = fminf(fmaxf(1024.f * sp / (0.125f * sum), 512.f), 2048.f);
        w = (uint32_t)(0.5f * ((float)w + want));
        w = w < 512u ? 512u : w > 2048u ? 2048u : w;
        __hip_atomic_store(&g_xcd_w[x], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      xb[x] = w;
    }
  }
  // the gated fallback's threshold table, over ITS padded batch (kernel 6 / 8 / 9 pad to 256 / 128 / 128
  // queries, which can exceed this launch's nq_pad: the grid covers both)
  if (ftau && q < ftau_nq && lane < kFallbackTauW) ftau[(int64_t)q * kFallbackTauW + lane] = 0u;
  if (q >= nq_pad) return;
  if (lane < k10::kTauW) tau[(int64_t)q * k10::kTauW + lane] = 0u;
  float y[NM][4];
  float am = 0.f;
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    if constexpr (DT == RFX_F32) {
      float4 v = float4{0.f, 0.f, 0.f, 0.f};
      if (q < nq) v = *(const float4*)((const float*)Q + (int64_t)q * D + 256 * m + 4 * lane);
      y[m][0] = v.x;
      y[m][1] = v.y;
      y[m][2] = v.z;
      y[m][3] = v.w;
    } else {
      uint2 v = uint2{0u, 0u};
      if (q < nq) v = *(const uint2*)((const uint16_t*)Q + (int64_t)q * D + 256 * m + 4 * lane);
      const uint32_t u[2] = {v.x, v.y};
#pragma unroll
      for (int e = 0; e < 4; ++e) y[m][e] = widen<DT>((uint16_t)(e & 1 ? u[e >> 1] >> 16 : u[e >> 1] & 0xffffu));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(y[m][e]));
  }
  am = wave_max_f32(am);  // DPP + readlane, no ds_bpermute round trips (rfx_device.h)
  const float s = am > 0.f ? __fdiv_rn(am, 127.f) : 0.f;
  double ey = 0.0;
  int cc = 0;  // <= D 127^2 < 2^31
  uint32_t pkm[NM];  // (the seed below reads them back)
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    uint32_t pk = 0u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int8_t c = s > 0.f ? code_of(y[m][e], s) : (int8_t)0;
      pk |= (uint32_t)(uint8_t)c << (8 * e);
      const double d = (double)y[m][e] - (double)s * (double)c;
      ey += d * d;
      cc += (int)c * c;
    }
    *(uint32_t*)(Qc + (int64_t)q * D + 256 * m + 4 * lane) = pk;
    pkm[m] = pk;
  }
  ey = wave_sum_f64(ey);
  cc = wave_sum_i32(cc);
  if (seed && (X8 == nullptr || kl <= 0)) {
    if (lane == 0) seed[q] = 0u;  // (no seed: kernel 10 starts with no bound)
  } else if (seed) {
    // the seed: 16 lanes per sample row (lane gl holds 16-B chunks gl + 16 u of the row and of the query codes,
    // gathered from the lanes that hold them: lane l has bytes 256 m + 4 l .. + 3), 4 rows per group in flight
    constexpr int NU = D / 256;
    __shared__ float sv[4][kSeedRows];
    const int wv = threadIdx.x >> 6, g = lane >> 4, gl = lane & 15;
    uint4 qd[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      qd[u].x = __shfl(pkm[u], 4 * gl + 0);
      qd[u].y = __shfl(pkm[u], 4 * gl + 1);
      qd[u].z = __shfl(pkm[u], 4 * gl + 2);
      qd[u].w = __shfl(pkm[u], 4 * gl + 3);
    }
    const int S = nrows < kSeedRows ? nrows : kSeedRows;
    for (int i0 = 0; i0 < S; i0 += 16) {
      uint4 xv[4][NU];
      int rr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = i0 + 4 * g + t;
        rr[t] = (int)((int64_t)(i < S ? i : 0) * nrows / S);
#pragma unroll
        for (int u = 0; u < NU; ++u) xv[t][u] = *(const uint4*)(X8 + (int64_t)rr[t] * D + 16 * (gl + 16 * u));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        int acc = 0;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          acc = __builtin_amdgcn_sdot4((int)xv[t][u].x, (int)qd[u].x, acc, false);
          acc = __builtin_amdgcn_sdot4((int)xv[t][u].y, (int)qd[u].y, acc, false);
          acc = __builtin_amdgcn_sdot4((int)xv[t][u].z, (int)qd[u].z, acc, false);
          acc = __builtin_amdgcn_sdot4((int)xv[t][u].w, (int)qd[u].w, acc, false);
        }
        const float dsum = row16_sum((float)acc);  // |partial sums| < 2^24: exact in f32
        const int i = i0 + 4 * g + t;
        if (gl == 0 && i < S) {
          const uint4 md = tmeta[rr[t] >> 5];
          const int r = rr[t];
          const bool ok = ((md.y >> (r & 31)) & 1u) && (mask == nullptr || ((mask[r >> 5] >> (r & 31)) & 1u));
          sv[wv][i] = ok ? dsum * __uint_as_float(md.x) : -__builtin_inff();  // A = s_t D, one rounding
        }
      }
    }
    // the KL-th best of the S values (4 per lane, sorted; kl rounds of a wave max)
    float a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = 64 * j + lane < S ? sv[wv][64 * j + lane] : -__builtin_inff();
    auto cx = [](float& x, float& y) {
      const float hi = fmaxf(x, y), lo = fminf(x, y);
      x = hi;
      y = lo;
    };
    cx(a[0], a[1]);
    cx(a[2], a[3]);
    cx(a[0], a[2]);
    cx(a[1], a[3]);
    cx(a[1], a[2]);
    float mx = -__builtin_inff();
    for (int it = 0; it < kl; ++it) {
      mx = wave_max_f32(a[0]);
      const bool win = lane == (int)__builtin_ctzll(__ballot(a[0] == mx));
      a[0] = win ? a[1] : a[0];
      a[1] = win ? a[2] : a[1];
      a[2] = win ? a[3] : a[2];
      a[3] = win ? -__builtin_inff() : a[3];
    }
    if (lane == 0) seed[q] = (q < nq && mx > -__builtin_inff()) ? ord(mx) : 0u;
  }
  if (lane == 0) {
    float e2 = 0.f;
    if (s > 0.f) {
      const double xm = (double)__uint_as_float(stats[0]), em = (double)__uint_as_float(stats[1]);
      const double yh = (double)s * sqrt((double)cc);
      const double eq = xm * sqrt(ey) + em * yh;
      e2 = f32_up((2.0 * eq + 4e-7 * (xm + em) * yh + 2.4e-7 * xm * (yh + sqrt(ey))) * (1.0 + 1e-5) / (double)s);
    }
    qe2[q] = e2;
  }
}

// ---- select: survivors, exact re-score, top-k (one 512-thread block per query; k_select.h) ----------
template <int DT, int D>
__global__ __launch_bounds__(512) void screen_select_kernel(const float* __restrict__ cs, const int* __restrict__ cr,
                                                            const uint32_t* __restrict__ drops, int64_t n_lists,
                                                            int list_len, const float* __restrict__ qe2,
                                                            const uint8_t* __restrict__ Q,
                                                            const uint8_t* __restrict__ X, int k, int64_t row_offset,
                                                            float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                                            sel::Rec* __restrict__ out_rec, uint32_t* __restrict__ gate,
                                                            int* __restrict__ diag, int force) {
  __shared__ sel::SelLds sl;
  sel::select_body<DT, D>(cs, cr, drops, n_lists, list_len, qe2, Q, X, k, row_offset, out_s, out_r, out_rec, gate, diag,
                          force, (int64_t)blockIdx.x, sl);
}

}  // namespace

#ifdef RFX_DEBUG_BUILD
int dbg_select_times(unsigned long long* out_h) {
  return hipMemcpyFromSymbol(out_h, HIP_SYMBOL(g_sel_t), sizeof(g_sel_t)) == hipSuccess ? 0 : -1;
}
#endif

// ---- host launchers --------------------------------------------------------------------------------
// the int8 copy: bf16 / f16 / f32 stores at d 768 / 1024 (kernel 10 screens bf16 / f16 batches,
// kernel 11 a few questions of any of the three)
bool screen_supported(int D, int dtype) {
  return (D == 768 || D == 1024) && (dtype == RFX_BF16 || dtype == RFX_F16 || dtype == RFX_F32);
}

void launch_screen_quantize(const void* X, int D, int dtype, int64_t tile0, int64_t ntiles, const int64_t* tiles_d,
                            int8_t* codes, void* tmeta, uint32_t* stats, hipStream_t st) {
  if (ntiles <= 0) return;
#define RFX_SQ(DTV, DV)                                                                                         \
  hipLaunchKernelGGL((screen_quantize_kernel<DTV, DV>), dim3((unsigned)ntiles), dim3(256), 0, st, X, \
                     tile0, tiles_d, codes, (uint4*)tmeta, stats)
  if (dtype == RFX_BF16 && D == 768)
    RFX_SQ(RFX_BF16, 768);
  else if (dtype == RFX_BF16)
    RFX_SQ(RFX_BF16, 1024);
  else if (dtype == RFX_F32 && D == 768)
    RFX_SQ(RFX_F32, 768);
  else if (dtype == RFX_F32)
    RFX_SQ(RFX_F32, 1024);
  else if (D == 768)
    RFX_SQ(RFX_F16, 768);
  else
    RFX_SQ(RFX_F16, 1024);
#undef RFX_SQ
}

// Batches of up to 64 questions (the micro-batches of rfx/batcher.py: <= 50 chat threads per process,
// config.py:137, chat.py:496-521) run the 2-wave kernel: 64 queries per workgroup, two workgroups per CU,
// 512 workgroups over the corpus (fewer on a small store: >= 8 tiles each).  Larger batches the 8-wave
// kernel (256 queries per workgroup, one per CU).  RFX_SCREEN_W2_BLOCKS (tuning) overrides the former's count.
// RFX_K10_Q64=1: batches of more than 64 questions at d 768 run the 64-queries-per-wave kernel
// (k_scan_screen64.h: 4 waves x 64 queries, one list per query per workgroup) instead of the 8-wave one
bool screen_q64() {
  static const bool v = [] {
    const char* e = getenv("RFX_K10_Q64");
    return e && e[0] == '1';
  }();
  return v;
}

int screen_w2_blocks() {
  static const int v = [] {
    const char* e = getenv("RFX_SCREEN_W2_BLOCKS");
    return e && *e ? atoi(e) : 0;
  }();
  return v;
}

MfmaPlan plan_scan_screen(int64_t nrows, int D, int dtype, int64_t nq, int k, int max_blocks) {
  MfmaPlan p{};
  p.ok = screen_supported(D, dtype) && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : -1);
  if (p.k_lane < 0) p.ok = false;
  const bool w2 = nq <= k10::kQGSmall;
  p.bn = w2 ? k10::kQGSmall : k10::kQG;
  p.q_blocks = (int)((nq + p.bn - 1) / p.bn);
  p.nq_pad = (int64_t)p.q_blocks * p.bn;
  if (p.q_blocks < 1 || p.q_blocks > 256) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k10::kTM - 1) / k10::kTM, 1);
  int64_t ranges;
  if (w2) {
    ranges = max_blocks > 0 ? max_blocks : screen_w2_blocks() > 0 ? screen_w2_blocks() : 512;
    // >= ~12 tiles per workgroup: each block's first tiles pass nearly every value (its bound is not there
    // yet), so a small store wants fewer, longer blocks (100k x 768 f32, nq 32: 256 blocks 0.079 ms, 384
    // blocks 0.104 ms, 128 blocks 0.082 ms; profiles/r06/tune/)
    ranges = std::min<int64_t>(ranges, std::max<int64_t>(ntiles / 12, 8));
    if (ranges > 8) ranges = ranges / 8 * 8;  // (a multiple of 8: the XCD-balanced split)
  } else {
    ranges = std::max<int64_t>((max_blocks > 0 ? max_blocks : 256) / std::max(p.q_blocks, 1), 1);
  }
  ranges = std::max<int64_t>(std::min<int64_t>(ranges, ntiles), 1);
  p.blocks = (int)ranges;
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.lists_per_block = (!w2 && D == 768 && screen_q64()) ? 1 : 2;  // (the 64-queries-per-wave kernel: one list)
  p.n_lists = (int64_t)p.blocks * p.lists_per_block;
  return p;
}

// the slot table [nq_pad][16], then kernel 10's XCD-split words (k10::kXbWords), then the seeds [nq_pad]
size_t tau_bytes_screen(const MfmaPlan& p) {
  return ((size_t)p.nq_pad * k10::kTauW + k10::kXbWords + (size_t)p.nq_pad) * sizeof(uint32_t);
}

uint32_t* xcd_weights_device_ptr() {
  static uint32_t* ptr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!ptr[dev] && hipGetSymbolAddress((void**)&ptr[dev], HIP_SYMBOL(g_xcd_w)) != hipSuccess) ptr[dev] = nullptr;
  return ptr[dev];
}

void launch_screen_queries(const void* Q, int dtype, int D, int64_t nq, int64_t nq_pad, int8_t* Qc, float* qe2,
                           const uint32_t* stats, uint32_t* tau, uint32_t* gate, uint32_t* ftau, int64_t ftau_nq,
                           hipStream_t st, const ScreenSeed* sd) {
  if (!ftau) ftau_nq = 0;
  const dim3 grid((unsigned)((std::max(nq_pad, ftau_nq) + 3) / 4));
  // the seed words follow the slot table and the XCD words (tau_bytes_screen).  Off by default: measured
  // no faster; RFX_K10_SEED=1 computes it (A/B), otherwise the quantiser writes zeros.
  static const bool seed_on = [] {
    const char* e = getenv("RFX_K10_SEED");
    return e && e[0] == '1';
  }();
  uint32_t* seed = tau + nq_pad * k10::kTauW + k10::kXbWords;
  const bool use = sd && sd->X8 && sd->nrows > 0 && seed_on;
#define RFX_SQQ(DTV, DV)                                                                                       \
  hipLaunchKernelGGL((screen_queries_kernel<DTV, DV>), grid, dim3(256), 0, st, Q, (int)nq, (int)nq_pad, Qc, qe2,  \
                     stats, tau, gate, ftau, (int)ftau_nq, tau + nq_pad * k10::kTauW, use ? sd->X8 : nullptr,      \
                     use ? (const uint4*)sd->tmeta : nullptr, use ? sd->nrows : 0, use ? sd->mask : nullptr,       \
                     use ? sd->kl : 0, seed)
  if (dtype == RFX_BF16 && D == 768)
    RFX_SQQ(RFX_BF16, 768);
  else if (dtype == RFX_BF16)
    RFX_SQQ(RFX_BF16, 1024);
  else if (dtype == RFX_F32 && D == 768)
    RFX_SQQ(RFX_F32, 768);
  else if (dtype == RFX_F32)
    RFX_SQQ(RFX_F32, 1024);
  else if (D == 768)
    RFX_SQQ(RFX_F16, 768);
  else
    RFX_SQQ(RFX_F16, 1024);
#undef RFX_SQQ
}

int launch_scan_screen(const MfmaPlan& p, const int8_t* codes, const void* tmeta, const uint32_t* stats, int nrows, int D,
                       const int8_t* Qc, const float* qe2, int nq, uint32_t* tau, float* cs, int* cr, uint32_t* drops,
                       hipStream_t st, const uint32_t* mask) {
  if (!p.ok || (D != 768 && D != 1024)) return -1;
  const int ntiles = (nrows + k10::kTM - 1) / k10::kTM;
  dim3 grid(p.blocks, p.q_blocks);
  auto f = p.bn == k10::kQGSmall ? (D == 768 ? k10::launch_768_w2 : k10::launch_1024_w2)
           : p.lists_per_block == 1 ? k10q::launch_768
                                    : (D == 768 ? k10::launch_768 : k10::launch_1024);
  return f(p.k_lane, grid, st, codes, (const uint4*)tmeta, stats, Qc, qe2, nq, ntiles, tau, cs, cr, drops, p.n_lists,
           mask, tau + p.nq_pad * k10::kTauW, xcd_weights_device_ptr());
}

int launch_screen_select(const float* cs, const int* cr, const uint32_t* drops, int64_t n_lists, int list_len,
                         const float* qe2, const void* Q, const void* X, int D, int dtype, int64_t nq, int k,
                         int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec, uint32_t* gate, int* diag,
                         int force, hipStream_t st) {
  if (nq <= 0) return 0;
  if (k < 1 || k > sel::kSelK) return -1;
#define RFX_SEL(DTV, DV)                                                                                          \
  hipLaunchKernelGGL((screen_select_kernel<DTV, DV>), dim3((unsigned)nq), dim3(512), 0, st, cs, cr, drops, n_lists, \
                     list_len, qe2, (const uint8_t*)Q, (const uint8_t*)X, k, row_offset, out_s, out_r,             \
                     (sel::Rec*)out_rec, gate, diag, force)
  if (dtype == RFX_BF16 && D == 768)
    RFX_SEL(RFX_BF16, 768);
  else if (dtype == RFX_BF16)
    RFX_SEL(RFX_BF16, 1024);
  else if (dtype == RFX_F32 && D == 768)
    RFX_SEL(RFX_F32, 768);
  else if (dtype == RFX_F32)
    RFX_SEL(RFX_F32, 1024);
  else if (D == 768)
    RFX_SEL(RFX_F16, 768);
  else
    RFX_SEL(RFX_F16, 1024);
#undef RFX_SEL
  return 0;
}

}  // namespace rfx
