// k_select_fb.h — the two-pass scan's select with its exact fallback inside the same launch (bf16 / f16 at
// d 768, the fallback plan of kernel 6).  DESIGN §4.10c "Fewer launches".
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551); one batch of
// the micro-batcher or one rank's shard of a multi-GPU search.
// Before this kernel a search ran the select, then kernel 6 over every row and the merge of its lists, both
// gated on a device word the select sets when some query's survivors may be incomplete: two launches that
// returned at once in nearly every search and still cost ~11 us of the 8-GPU shard's step.  Here the select's
// workgroups go on to those two steps themselves when the word is set:
//   1. select: each workgroup CLAIMS queries from a counter and selects them (k_select.h); a query that
//      cannot be proven is marked (diag 2 q + 1 = -1) and sets the gate;
//   2. a workgroup whose claims ran out leaves if the gate is clear; the one that made the last selects-done
//      count reads the final gate, so it stays whenever the gate is set.  Workgroups that stay wait until every query is
//      selected, then claim kernel 6's workgroups (row range, query group) as units and run its body in
//      their LDS, then, once every unit is done, claim queries and merge the marked ones' lists (merge_one
//      + rescore_final: the bits the separate merge launch wrote).  The other queries keep the select's answer.
// No co-residency of the grid is needed: a workgroup waits only for work that is already claimed, i.e. held
// by a running workgroup, and the one that finishes the last select always stays when the gate is set, so
// the fallback completes with whichever workgroups take part.  Proven and marked queries are written by
// different steps (no two writers of one answer).  The waits are bounded (kMaxPolls): a wait that runs out
// (never expected) sets the error word and lets the workgroup go on.
// Control words (the search's 256-B gate area, zeroed by the query quantiser each search): below.
#pragma once
#include "k_scan_mfma6.h"
#include "k_scan_valu.h"
#include "k_select.h"

namespace rfx {
namespace selfb {

constexpr int kWGate = 0;        // set by a select that cannot prove its query
constexpr int kWSelClaim = 8;    // queries claimed
constexpr int kWSelDone = 16;    // queries selected
constexpr int kWUnitClaim = 24;  // kernel-6 units claimed
constexpr int kWUnitDone = 32;   // kernel-6 units done
constexpr int kWMergeClaim = 40; // queries claimed by the merge
constexpr int kWErr = 48;        // a wait ran out (never expected)
constexpr uint32_t kMaxPolls = 1u << 22;  // x s_sleep 8 (~0.5 us): about 2 s

// One claim for the workgroup (uniform: readfirstlane of the LDS word, see kernel 11's claim loop)
__device__ __forceinline__ int claim(uint32_t* ctr, int* slot) {
  if (threadIdx.x == 0) *slot = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int v = __builtin_amdgcn_readfirstlane(*slot);
  __syncthreads();  // (the slot is reused by the next claim)
  return v;
}

// Wait until ctl[wd] >= target, then acquire: the workgroup sees what the counted work wrote.
__device__ __forceinline__ void wait_count(uint32_t* ctl, int wd, uint32_t target) {
  if (threadIdx.x == 0) {
    for (uint32_t i = 0;; ++i) {
      if (__hip_atomic_load(ctl + wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if (i >= kMaxPolls) {
        __hip_atomic_store(ctl + kWErr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

template <int DT, int KL, int MODE>
__global__ __launch_bounds__(512, 1) void select_fb_kernel(SelectFb a) {
  constexpr int D = 768;
  constexpr int K = KL <= 4 ? 4 : 16;  // the merge's list slot (valu_k_slot of k <= KL)
  __shared__ __attribute__((aligned(1024))) uint8_t lds[k6::lds_bytes<KL, k6::kRing>()];
  static_assert(sizeof(sel::SelLds) <= k6::lds_bytes<KL, k6::kRing>(), "the select's LDS lies in kernel 6's");
  __shared__ int slot;
  sel::SelLds& sl = *reinterpret_cast<sel::SelLds*>(lds);
  uint32_t* const ctl = a.ctl;
  const int nq = (int)a.nq, tid = threadIdx.x;
  const uint8_t* const Q = (const uint8_t*)a.Qpad;
  // 1. the select, one claimed query at a time (at most nq claims per workgroup)
  for (int it = 0; it <= nq; ++it) {
    const int q = claim(ctl + kWSelClaim, &slot);
    if (q >= nq) break;
    sel::select_body<DT, D>(a.cs, a.cr, a.drops, a.n_lists, a.list_len, a.qe2, Q, (const uint8_t*)a.X, a.k,
                            a.row_offset, a.out_s, a.out_r, (sel::Rec*)a.out_rec, ctl + kWGate, a.diag, a.force,
                            (int64_t)q, sl);
    __syncthreads();  // (the LDS is reused by the next query)
    if (tid == 0) {
      // the mark (diag) and the gate written by this thread reach the agent before the count
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(ctl + kWSelDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // 2. leave unless the gate is set.  Read after this workgroup's last count: the workgroup that made the
  // last count (its RMW follows every other count, each released after its gate store) sees the final gate.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const uint32_t g = __hip_atomic_load(ctl + kWGate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__builtin_amdgcn_readfirstlane(g) == 0u) return;
  wait_count(ctl, kWSelDone, (uint32_t)nq);
  // 3. kernel 6 over every row, unit u = (row range u % blocks, query group u / blocks)
  const int units = a.mp.blocks * a.mp.q_blocks;
  const int ntiles = (a.nrows + k6::kTM - 1) / k6::kTM;
  for (int it = 0; it <= units; ++it) {
    const int u = claim(ctl + kWUnitClaim, &slot);
    if (u >= units) break;
    k6::scan_mfma6_body<DT, KL, D, MODE>((const uint16_t*)a.X, (const uint16_t*)a.Qpad, nq, ntiles, a.tau, a.fcs,
                                         a.fcr, a.mp.n_lists, a.mask, u % a.mp.blocks, u / a.mp.blocks, a.mp.blocks,
                                         lds);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every lane's list stores
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(ctl + kWUnitDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  wait_count(ctl, kWUnitDone, (uint32_t)units);
  // 4. the merge of the marked queries' lists (the separate merge launch's K, lists and re-score)
  const FlatSrc<false> src{a.fcs, a.fcr, a.n_cand};
  for (int it = 0; it <= nq; ++it) {
    const int q = claim(ctl + kWMergeClaim, &slot);
    if (q >= nq) break;
    const int mark = __hip_atomic_load(a.diag + 2 * (int64_t)q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(mark) != -1) continue;
    merge_one<K, false, 8, true>(src, (int64_t)q, a.mp.k_lane, a.k, a.row_offset, a.out_s, a.out_r,
                                 (MergeRec*)a.out_rec);
    if (a.rs.X) rescore_final(a.rs, (int64_t)q, a.k, a.row_offset, a.out_s, a.out_r, (MergeRec*)a.out_rec);
    __syncthreads();
  }
}

// one translation unit per dtype (kselfb_*.hip): KL 4 / 10, with and without the row mask
#define RFX_SELFB_INSTANTIATE(DTV, NAME)                                                                      \
  int NAME(const SelectFb& a, hipStream_t st) {                                                               \
    const int units = a.mp.blocks * a.mp.q_blocks;                                                            \
    const dim3 grid((unsigned)std::max<int64_t>(a.nq, std::min(units, 256)));                                 \
    if (a.mp.k_lane == 4 && !a.mask)                                                                          \
      hipLaunchKernelGGL((select_fb_kernel<DTV, 4, 0>), grid, dim3(512), 0, st, a);                           \
    else if (a.mp.k_lane == 10 && !a.mask)                                                                    \
      hipLaunchKernelGGL((select_fb_kernel<DTV, 10, 0>), grid, dim3(512), 0, st, a);                          \
    else if (a.mp.k_lane == 4)                                                                                \
      hipLaunchKernelGGL((select_fb_kernel<DTV, 4, k6::kModeMask>), grid, dim3(512), 0, st, a);               \
    else if (a.mp.k_lane == 10)                                                                               \
      hipLaunchKernelGGL((select_fb_kernel<DTV, 10, k6::kModeMask>), grid, dim3(512), 0, st, a);              \
    else                                                                                                      \
      return -1;                                                                                              \
    return 0;                                                                                                 \
  }

}  // namespace selfb
}  // namespace rfx
