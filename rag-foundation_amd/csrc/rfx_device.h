// rfx_device.h — device-side helpers shared by the gfx950 kernels.
// CDNA4 only: wave64, DPP row ops, MFMA builtins.  No CUDA-compat layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rfx {

constexpr int kWave = 64;
constexpr int kEmptyRow = 0x7fffffff;  // internal "no row" sentinel (worst under the tie rule)

// ---- ranking rule: score desc, then row asc -------
// NaN scores (tombstoned rows) never compare better than anything, so they are never kept.
__device__ __forceinline__ bool better(float s1, int r1, float s2, int r2) {
  return s1 > s2 || (s1 == s2 && r1 < r2);
}
__device__ __forceinline__ bool better64(float s1, long long r1, float s2, long long r2) {
  return s1 > s2 || (s1 == s2 && r1 < r2);
}

// orderable u32 of a non-NaN float (larger float -> larger key; 0 stays below every score key)
__device__ __forceinline__ uint32_t ord_f32(float s) {
  const uint32_t u = __float_as_uint(s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ---- row masks (metadata filters): bit (r & 31) of word r >> 5 set = row r may be returned ------
// A lane of a 32x32 MFMA accumulator holds rows rb + (r & 3) + 8 (r >> 2), r < 16, with
// rb ≡ 0 or 4 (mod 32): all in word rb >> 5.  acc_row_bits puts row (r & 3) + 8 (r >> 2) of the
// lane at that bit; words past the mask (rows past the end, NaN anyway) read as 0.
__device__ __forceinline__ uint32_t acc_row_bits(const uint32_t* __restrict__ mask, int rb, int nrows) {
  const int w = rb >> 5;
  return w < ((nrows + 31) >> 5) ? mask[w] >> (rb & 31) : 0u;
}
// masked-out rows become NaN, which no top-k compare admits (the tombstone rule)
template <class V>
__device__ __forceinline__ void mask_acc16(V& acc, uint32_t bits) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (!((bits >> ((r & 3) + 8 * (r >> 2))) & 1u)) acc[r] = __builtin_nanf("");
}
__device__ __forceinline__ bool row_allowed(const uint32_t* __restrict__ mask, int row) {
  return (mask[row >> 5] >> (row & 31)) & 1u;
}

// ---- counter-based generator (oracle/synth.py restates this bit-for-bit) ----------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// odd integer in (-2^24, 2^24) of generator key idx (oracle/synth.py raw_rows)
__device__ __forceinline__ int32_t synth_raw(uint64_t base, uint64_t idx) {
  const uint64_t u = splitmix64(base + idx);
  return (int32_t)(2u * (uint32_t)(u >> 40)) + 1 - (1 << 24);
}

// ---- fp32 <-> 16-bit storage -----------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even; NaN stays NaN (quiet)
__host__ __device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  return (float)__builtin_bit_cast(_Float16, h);
}
// The asm barrier pins the f32 value: without it LLVM folds an f64->f32->f16 chain into a single
// f64->f16 rounding, which differs from the two-step rounding the oracle (numpy) performs.
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  asm volatile("" : "+v"(f));
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

// ---- cross-lane -------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// sum over each DPP row of 16 lanes; every lane of the row receives the row sum.
// row_ror:n (0x120+n) rotates within the 16-lane row.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}

// Wave reductions without ds_bpermute: a __shfl_xor is an LDS-crossbar round trip (~100 cycles with
// its wait), six of them per reduction.  DPP row_ror within each 16-lane row (every lane receives
// its row's result), then the four row results by readlane; every lane receives the wave's result.
// For lane 0 of a row, row_ror in the order 8, 4, 2, 1 pairs the same partial sums as a xor
// butterfly in that order, so row16_sum_f64's lane-0 sum equals the __shfl_xor version bit for bit.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xf, 0xf, false));
  const uint32_t a = __builtin_amdgcn_readlane((int)v, 0), b = __builtin_amdgcn_readlane((int)v, 16);
  const uint32_t c = __builtin_amdgcn_readlane((int)v, 32), d = __builtin_amdgcn_readlane((int)v, 48);
  return max(max(a, b), max(c, d));
}
__device__ __forceinline__ float wave_max_f32(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, false)));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}
__device__ __forceinline__ double row16_sum_f64(double v) {
#define RFX_DPP_F64_STEP(ctl)                                                                       \
  {                                                                                                 \
    const long long b = __double_as_longlong(v);                                                    \
    const int lo = __builtin_amdgcn_mov_dpp((int)b, ctl, 0xf, 0xf, false);                          \
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), ctl, 0xf, 0xf, false);                  \
    v += __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));          \
  }
  RFX_DPP_F64_STEP(0x128)
  RFX_DPP_F64_STEP(0x124)
  RFX_DPP_F64_STEP(0x122)
  RFX_DPP_F64_STEP(0x121)
#undef RFX_DPP_F64_STEP
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
  v = row16_sum_f64(v);
  const long long b = __double_as_longlong(v);
  double s = 0.0;
#pragma unroll
  for (int r = 0; r < 64; r += 16) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)b, r), hi = __builtin_amdgcn_readlane((int)(b >> 32), r);
    s += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  }
  return s;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x122, 0xf, 0xf, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x121, 0xf, 0xf, false);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

// lane l receives lane l-1's value (lane 0 keeps its own): one DPP move (wave_shr:1, GFX9 DPP)
// instead of a ds_bpermute round trip through the LDS crossbar — the list insert's critical path.
__device__ __forceinline__ int lane_shr1(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ float lane_shr1(float v) { return __int_as_float(lane_shr1(__float_as_int(v))); }
__device__ __forceinline__ long long lane_shr1(long long v) {
  const int lo = lane_shr1((int)v), hi = lane_shr1((int)(v >> 32));
  return (long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ---- wave-resident top-K list ------------------------------------------------------------------
// The list lives in lanes 0..K-1 of (ls, lr), best first; empty slots are (-inf, kEmptyRow).
// Candidates arrive one per lane; those that beat the wave-uniform threshold (entry K-1) are
// inserted one at a time (ballot + popcount for the position, one DPP lane shift).
template <int K>
struct WaveList {
  float ls;
  int lr;
  float ts;  // threshold = entry K-1 (wave-uniform)
  int tr;

  __device__ __forceinline__ void init() {
    ls = -__builtin_inff();
    lr = kEmptyRow;
    ts = -__builtin_inff();
    tr = kEmptyRow;
  }

  __device__ __forceinline__ void offer(float cs, int cr, bool valid) {
    const int lane = lane_id();
    uint64_t mask = __ballot(valid && better(cs, cr, ts, tr));
    while (mask) {
      const int j = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float s = readlane_f(cs, j);
      const int r = readlane_i(cr, j);
      if (!better(s, r, ts, tr)) continue;  // wave-uniform: threshold may have risen
      const bool b = (lane < K) && better(ls, lr, s, r);
      const int pos = __popcll(__ballot(b));
      const float us = lane_shr1(ls);
      const int ur = lane_shr1(lr);
      if (lane > pos && lane < K) {
        ls = us;
        lr = ur;
      }
      if (lane == pos) {
        ls = s;
        lr = r;
      }
      ts = readlane_f(ls, K - 1);
      tr = readlane_i(lr, K - 1);
    }
  }
};

// Same with 64-bit row ids (cross-shard merge of global rows).
template <int K>
struct WaveList64 {
  float ls;
  long long lr;
  float ts;
  long long tr;
  float fs;  // admission floor (wave-uniform): the threshold never drops below it
  long long fr;

  __device__ __forceinline__ void init() {
    ls = -__builtin_inff();
    lr = 0x7fffffffffffffffll;
    ts = fs = -__builtin_inff();
    tr = fr = 0x7fffffffffffffffll;
  }

  // empty list whose admission threshold is (s, r): only strictly better candidates enter, also
  // after inserts (the threshold is max(floor, entry K-1), so an empty tail cannot lower it)
  __device__ __forceinline__ void init_above(float s, long long r) {
    init();
    ts = fs = s;
    tr = fr = r;
  }

  __device__ __forceinline__ void offer(float cs, long long cr, bool valid) {
    const int lane = lane_id();
    uint64_t mask = __ballot(valid && better64(cs, cr, ts, tr));
    while (mask) {
      const int j = __builtin_ctzll(mask);
      mask &= mask - 1;
      const float s = readlane_f(cs, j);
      const long long r = (long long)(((uint64_t)(uint32_t)readlane_i((int)(cr >> 32), j) << 32) |
                                      (uint32_t)readlane_i((int)cr, j));
      if (!better64(s, r, ts, tr)) continue;
      const bool b = (lane < K) && better64(ls, lr, s, r);
      const int pos = __popcll(__ballot(b));
      const float us = lane_shr1(ls);
      const long long ur = lane_shr1(lr);
      if (lane > pos && lane < K) {
        ls = us;
        lr = ur;
      }
      if (lane == pos) {
        ls = s;
        lr = r;
      }
      const float ks = readlane_f(ls, K - 1);
      const long long kr = (long long)(((uint64_t)(uint32_t)readlane_i((int)(lr >> 32), K - 1) << 32) |
                                       (uint32_t)readlane_i((int)lr, K - 1));
      const bool above = better64(ks, kr, fs, fr);
      ts = above ? ks : fs;
      tr = above ? kr : fr;
    }
  }
};

}  // namespace rfx
