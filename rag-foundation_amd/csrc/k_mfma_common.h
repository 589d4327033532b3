// k_mfma_common.h — device helpers shared by the MFMA scan kernels (k_scan_mfma3/4/5.h): MFMA
// wrappers, orderable score keys, LDS-DMA / buffer-atomic inline asm, the shared pruning-bound
// table reads and the per-lane top-k list fold.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
#pragma once
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {
namespace mfc {

typedef __attribute__((ext_vector_type(8))) __bf16 v4bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 v4f16x8;
typedef __attribute__((ext_vector_type(16))) float v4f32x16;

template <int DT>
__device__ __forceinline__ v4f32x16 mfma(const uint4& a, const uint4& b, const v4f32x16& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v4bf16x8, a), __builtin_bit_cast(v4bf16x8, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v4f16x8, a), __builtin_bit_cast(v4f16x8, b), c,
                                                  0, 0, 0);
}

typedef __attribute__((ext_vector_type(4))) float v4f32x4;
template <int DT>
__device__ __forceinline__ v4f32x4 mfma16(const uint4& a, const uint4& b, const v4f32x4& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v4bf16x8, a), __builtin_bit_cast(v4bf16x8, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v4f16x8, a), __builtin_bit_cast(v4f16x8, b), c,
                                                  0, 0, 0);
}

__device__ __forceinline__ uint32_t ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// NaN-ignoring 3-way max.  Plain fmaxf (hipcc emits v_max3_f32): an inline-asm v_max3 reading an
// MFMA accumulator gets no MFMA->VALU wait states from hipcc and can read it before the MFMA has
// written it (measured: rows of a tile's first 8 accumulator registers lost, k_scan_mfma5.h).
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

typedef int v4i32 __attribute__((ext_vector_type(4)));

// Buffer descriptor (4 SGPRs) for a raw byte buffer at `base` (wave-uniform).
__device__ __forceinline__ v4i32 make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  v4i32 d;
  d.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  d.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xffff);  // stride 0
  d.z = -1;          // num_records: no range limit
  d.w = 0x00020000;  // raw dword buffer (gfx9 family)
  return d;
}
// LDS-DMA through a buffer descriptor: the lane address is base + 32-bit voff (one VGPR instead of
// a 64-bit address pair).  M0 = wave-uniform LDS destination; s_nop 4 covers a descriptor freshly
// written through v_readfirstlane (cdna_hip_programming.md §5.7 item 2).
__device__ __forceinline__ void bdma(v4i32 rsrc, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(lds_addr)
               : "memory", "m0");
}
// Same with the non-temporal hint (a stream read once: no reuse to keep in the caches).
__device__ __forceinline__ void bdma_nt(v4i32 rsrc, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff),
               "s"(rsrc), "s"(lds_addr)
               : "memory", "m0");
}
// Same at device scope (sc1: misses this CU's L1, sees other workgroups' atomics).
__device__ __forceinline__ void bdma_sc1(v4i32 rsrc, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc1 lds" ::"v"(voff),
               "s"(rsrc), "s"(lds_addr)
               : "memory", "m0");
}
// No-return device-scope unsigned max at rsrc + voff.  From asm, so hipcc neither waits for it nor
// reloads a 64-bit address for it; it joins the wave's vmcnt queue, which only makes the kernel's
// counted waits stricter (never looser).
__device__ __forceinline__ void batomic_umax(v4i32 rsrc, uint32_t voff, uint32_t val) {
  asm volatile("s_nop 4\n\tbuffer_atomic_umax %0, %1, %2, 0 offen" ::"v"(val), "v"(voff), "s"(rsrc) : "memory");
}

// LDS-DMA (global_load_lds_dwordx4) from inline asm; M0 = wave-uniform LDS destination.  The
// compiler cannot see a VMEM op writing LDS, so it does not drain the queue before LDS reads;
// the kernel orders them itself (counted vmcnt + s_barrier before a slot is read).
__device__ __forceinline__ void glds(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr)
               : "memory", "m0");
}
// Same, device scope (sc1): misses this CU's L1, so other workgroups' atomicMax updates of the
// threshold table are seen (a plain load may return an L1-resident stale line; stale stays exact).
__device__ __forceinline__ void glds_sc1(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(src), "s"(lds_addr)
               : "memory", "m0");
}

// Re-define registers through an empty asm.  Called on the resident query fragments right after the
// explicit s_waitcnt vmcnt(0) that lands them: hipcc's wait-count pass cannot see the asm LDS-DMA
// ops that share the vmcnt queue, so while it still tracks the fragments' loads it re-inserts
// s_waitcnt vmcnt(N) before their first use in EVERY tile (merging the loop back-edge with the
// preheader), and those waits drain the DMA ring (measured on kernel 10, round 3).
template <int N>
__device__ __forceinline__ void launder(uint4 (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    v4i32 t = __builtin_bit_cast(v4i32, v[i]);
    asm volatile("" : "+v"(t));
    v[i] = __builtin_bit_cast(uint4, t);
  }
}

// 16 values of four 16x16 accumulators as one flat vector (no copies)
struct Acc4View {
  const v4f32x4 (&a)[4];
  __device__ __forceinline__ float operator[](int r) const { return a[r >> 2][r & 3]; }
};

// min over the first KL threshold slots of one query (LDS image [q][kTauW] u32, 48 B per query)
template <int KL>
__device__ __forceinline__ uint32_t tau_min(const uint8_t* p) {
  const uint4 a = *(const uint4*)p;
  uint32_t m = min(min(a.x, a.y), min(a.z, a.w));
  if constexpr (KL > 4) {
    const uint4 b = *(const uint4*)(p + 16), c = *(const uint4*)(p + 32);
    m = min(m, min(min(b.x, b.y), min(b.z, b.w)));
    m = min(m, min(c.x, c.y));
  }
  return m;
}

// Fold one 32×32 accumulator (16 rows of one query per lane) into the lane's list.  The list lives
// in LDS (entry i of this lane at Ls[i * 64], best first).  One register per list holds the
// pruning bound thr_o = max(list's KL-th best, min of the shared slots) as an orderable score;
// both terms only grow, so the bound is kept as a running max.  The list is touched only when
// some row of the tile reaches the bound; after such an update the list's best is published to
// its slot (device atomicMax).
// ROWMAP 0: value r of the lane is row rbase + (r & 3) + 8 (r >> 2) (32x32 accumulator layout);
// ROWMAP 1: row rbase + (r & 7) + 16 (r >> 3) (the 16x16x32 pair-swapped layout of kernels 5, 6);
// ROWMAP 2: row rbase + (r & 3) + 16 (r >> 2) (four 16x16 row blocks of one query, kernel 7).
// V: anything with float operator[](int) over 16 values (a 32x32 accumulator, or Acc4View).
template <int KL, int ROWMAP = 0, class V = v4f32x16>
__device__ __forceinline__ void fold(const V& acc, uint64_t* Ls, uint32_t& thr_o, int rbase, v4i32 tau_rsrc,
                                     uint32_t slot_voff, int& n_slow) {
  float mx = max3f(acc[0], acc[1], acc[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) mx = max3f(mx, acc[r], acc[r + 1]);
  mx = fmaxf(mx, acc[15]);  // NaN-ignoring max
  const float thr = thr_o ? unord(thr_o) : -__builtin_inff();
  if (mx >= thr) {
    ++n_slow;
    // insert straight into the LDS list (few registers: this path runs while the resident query
    // fragments and both accumulators occupy nearly the whole register file)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float s = acc[r];
      if (s >= thr) {  // NaN (tombstoned rows, rows past the end) never passes
        const int row = ROWMAP == 0   ? rbase + (r & 3) + 8 * (r >> 2)
                        : ROWMAP == 1 ? rbase + (r & 7) + 16 * (r >> 3)
                                      : rbase + (r & 3) + 16 * (r >> 2);
        const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
        if (key > Ls[(KL - 1) * 64]) {
          int i = KL - 1;
          for (; i > 0; --i) {
            const uint64_t prev = Ls[(i - 1) * 64];
            if (prev >= key) break;
            Ls[i * 64] = prev;
          }
          Ls[i * 64] = key;
        }
      }
    }
    const uint32_t own = (uint32_t)(Ls[(KL - 1) * 64] >> 32);
    thr_o = own > thr_o ? own : thr_o;
    batomic_umax(tau_rsrc, slot_voff, (uint32_t)(Ls[0] >> 32));
  }
}

}  // namespace mfc
}  // namespace rfx
