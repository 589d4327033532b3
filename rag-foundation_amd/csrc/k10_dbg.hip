// k10_dbg.hip — DEBUG BUILD ONLY (librfx_dbg.so, `make dbg`): ablations and ring depths of the
// two-pass scan's int8 screen (k_scan_screen.h MODE bits: 1 no top-k fold, 2 no launder, 4 prefetch
// distance 1, 8 no corpus stream, 16 early slot-table refreshes, 32 slow-path entry count, 64 store-wide
// integer fast-path bound, 128 epilogue in place, 256 min-of-KL slot bound, 512 slow path never taken,
// 1024 serial LDS insert, 2048 slow-path issue priority, 4096 static tile split (no XCD balance),
// 8192 slow-path entries and trips per tile index, 32768 no stage barriers, 65536 per-block start / end
// wall clocks),
// 131072 epilogue after the stage-0 barrier, 262144 waves 4-7 one stage later (stagger), 524288 partner
// bound by v_permlane16_swap, 1048576 the round-5 u32-score fold (integer pass threshold, per-position
// inserts in tiles 0-1; slower, not production), 2097152 one wait + barrier per tile (RING 10 / 12; production
// at RING 10), 4194304 the slow path's float pass mask instead of the integer threshold, 16384 a sorted
// merge instead of the pop loop when some lane passes >= 8 values (round 5),
// 8388608 a list's best published only when it rose (round 5),
// via rfx_dbg_screen_variant; variant = 10^8 * RING + MODE (RING in {4, 6, 8, 10, 12}; round 5's first
// sessions used 10^7 * RING + MODE, rounds 3-4 100000 * RING + MODE).
#define RFX_K10_BLOCK_TIMES
#include "k_scan_screen64.h"

namespace rfx {
namespace k10q {
int launch_768(int kl, dim3 grid, hipStream_t st, const int8_t* X, const uint4* tm, const uint32_t* sts, const int8_t* Qc,
               const float* qe2, int nq, int ntiles, uint32_t* tau, float* cs, int* cr, uint32_t* dr, int64_t n_lists,
               const uint32_t* mask, uint32_t* xb, uint32_t* xw);
}  // namespace k10q

int launch_scan_screen_dbg(const MfmaPlan& p, int variant, const int8_t* X, const void* tmv, const uint32_t* sts,
                           int nrows, const int8_t* Qc, const float* qe2, int nq, uint32_t* tau, float* cs, int* cr,
                           uint32_t* dr, hipStream_t st) {
  const uint4* tm = (const uint4*)tmv;
  if (!p.ok || p.k_lane != 10) return -1;
  const int ntiles = (nrows + k10::kTM - 1) / k10::kTM;
  dim3 grid(p.blocks, p.q_blocks);
#define RFX_K10V(R, M)                                                                                        \
  case 100000000 * R + M:                                                                                          \
    hipLaunchKernelGGL((k10::scan_screen_kernel<10, 768, false, R, M>), grid, dim3(512), 0, st, X, tm, sts, Qc, \
                       qe2, nq, ntiles, tau, cs, cr, dr, p.n_lists, nullptr, tau + p.nq_pad * k10::kTauW,      \
                       xcd_weights_device_ptr());                                                             \
    break;
  switch (variant) {
    // (round 6 trimmed the list to the variants its tools run: production, no fold (1), no fold and no stream
    // (9), slow path never taken (512), the trips counter (8192) and the block clocks (65536); earlier rounds'
    // sweeps are in the profiles they wrote)
    RFX_K10V(10, 2097152 + 8388608)
    RFX_K10V(10, 2097152 + 8388608 + 1)
    RFX_K10V(10, 2097152 + 8388608 + 9)
    RFX_K10V(10, 2097152 + 8388608 + 512)
    RFX_K10V(10, 2097152 + 8388608 + 8192)
    RFX_K10V(10, 2097152 + 8388608 + 65536)
    RFX_K10V(10, 2097152 + 8388608 + 33554432)  // one wave DMAs the tile records (round 6 A/B)
    case 64:  // the 64-queries-per-wave kernel (k_scan_screen64.h; its plan: RFX_K10_Q64=1, one list per workgroup)
      if (p.lists_per_block != 1) return -1;
      return k10q::launch_768(10, grid, st, X, tm, sts, Qc, qe2, nq, ntiles, tau, cs, cr, dr, p.n_lists, nullptr,
                              tau + p.nq_pad * k10::kTauW, xcd_weights_device_ptr());
    case 65:  // the same, slow path never taken (timing)
    case 73:  // the same, no fold and no corpus stream (timing)
      if (p.lists_per_block != 1) return -1;
      if (variant == 65)
        hipLaunchKernelGGL((k10q::scan_screen_q64_kernel<10, 768, false, k10q::kRing768, 1>), grid, dim3(256), 0, st, X,
                           tm, sts, Qc, qe2, nq, ntiles, tau, cs, cr, dr, p.n_lists, nullptr, tau + p.nq_pad * k10::kTauW,
                           xcd_weights_device_ptr());
      else
        hipLaunchKernelGGL((k10q::scan_screen_q64_kernel<10, 768, false, k10q::kRing768, 9>), grid, dim3(256), 0, st, X,
                           tm, sts, Qc, qe2, nq, ntiles, tau, cs, cr, dr, p.n_lists, nullptr, tau + p.nq_pad * k10::kTauW,
                           xcd_weights_device_ptr());
      break;
    default:
      return -1;
  }
#undef RFX_K10V
  return 0;
}

int dbg_k10_trips(unsigned int* out_h, int reset) {
  if (reset) {
    static const unsigned int z[2][64] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(k10::g_k10_trips), z, sizeof(z)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out_h, HIP_SYMBOL(k10::g_k10_trips), sizeof(k10::g_k10_trips)) == hipSuccess ? 0 : -1;
}

int dbg_k10_block_times(unsigned long long* out_h) {
  return hipMemcpyFromSymbol(out_h, HIP_SYMBOL(k10::g_k10_bt), sizeof(k10::g_k10_bt)) == hipSuccess ? 0 : -1;
}

}  // namespace rfx
