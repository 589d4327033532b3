// rfx_kernels.h — host-side launchers of the gfx950 kernels (called by rfx_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/rfx.h"

namespace rfx {
// f64 re-score of a two-pass fallback's final top-k (k_scan_valu.h rescore_final)
struct Rescore {
  const void* X = nullptr;  // the index rows [rows][D] (dtype); nullptr = no re-score
  const void* Q = nullptr;  // the queries [nq][D] in the index dtype
  int D = 0;
  int dtype = 0;
  int64_t rows = 0;  // rows of X: an entry's row outside [row_offset, row_offset + rows) is padding
};

// ---- generator / maintenance -------------------------------------------------------------
void launch_synth_rows(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, void* out,
                       hipStream_t st);
void launch_nan_rows(void* X, const int64_t* rows_d, int64_t n, int64_t row_bytes, int dtype,
                     hipStream_t st);
void launch_stream_read(const void* p, int64_t bytes, uint32_t* out, hipStream_t st);
// also zeroes tau[0..n_tau) (the VALU scan's per-query pruning bounds) when tau != nullptr
void launch_widen_queries(const void* Q, int64_t n, int dtype, float* out, hipStream_t st, uint32_t* tau = nullptr,
                          int64_t n_tau = 0);

// ---- VALU scan (small nq) ------------------------------------------------------------------
struct ValuPlan {
  int vpr, vpl, k_slot, nqt, q_slices, rows_per_wave, blocks, n_lists;
  bool ok;
};
constexpr int kValuBlocks = 256;  // target workgroups of a VALU scan (one per CU; config-2 sweep)
int valu_k_slot(int k);
ValuPlan plan_scan_valu(int64_t nrows, int D, int dtype, int64_t nq, int k);
// mask (every scan launcher): optional row mask, bit (r & 31) of word r >> 5 set = row r may be
// returned, (nrows + 31) / 32 words; nullptr = all rows (the production kernels run unchanged).
// tau: optional [nq] u32 pruning bounds, zeroed beforehand (launch_widen_queries)
int launch_scan_valu(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const float* Qf,
                     int nq, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr,
                     uint32_t* tau = nullptr);
// The whole search (scan + final merge) in one launch for a VALU plan with nq <= kValuFusedMaxNq:
// Q is the raw [nq][D] query buffer in the index dtype; state = kValuFusedMaxNq bounds followed by
// p.q_slices arrival counters, ALL ZERO on entry — the kernel leaves them zero again, so a state
// buffer zeroed once serves every later search on one stream (rfx_api.hip keeps one per stream).
constexpr int kValuFusedMaxNq = 1024;
// + 160 words for the lone-question two-pass scan (kernel 11): counter, drops, fallback gate, and
// 16 bound slots for each of up to 8 queries
constexpr int kScreenValuState = kValuFusedMaxNq + 1024;
constexpr int kValuFusedStateWords = kScreenValuState + 160;
// gate (optional): the launch runs only when *gate != 0 (the two-pass scan's fallback)
int launch_search_valu_fused(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const void* Q, int nq,
                             float* cs, int* cr, uint32_t* state, int k, float* out_s, int64_t* out_r,
                             hipStream_t st, const uint32_t* mask = nullptr, const uint32_t* gate = nullptr);
// Kernel 11 (k_screen_valu.hip): the exact two-pass scan of nq <= 8 questions in one launch over the
// index's int8 copy (codes X8, tile records tmeta, quantiser stats), the exact rows X / queries Q in
// the index dtype; writes (out_s, out_r) and the fallback gate state[24] (state = the index's
// per-stream search state + kScreenValuState, zero on entry and left zero except the gate and the
// launch generation / verdict / claim words).  cx: [nq][blocks][16] u32 workspace, the exact score keys
// of the record entries (cs / cr) the blocks re-score.  For a lone question (screen_valu_inline_fallback) the
// exact fallback runs INSIDE the launch when the screen cannot prove its answer (vstate = the
// one-launch VALU search's state, the per-stream search state's base); otherwise the caller launches
// the gated one-launch VALU search after it (launch_search_valu_fused with gate = state + 24).
int launch_screen_valu(const ValuPlan& p, const int8_t* X8, const void* tmeta, const uint32_t* stats, int nrows, int D,
                       int dtype, const void* X, const void* Q, int nq, const uint32_t* mask, uint32_t* state,
                       uint32_t* vstate, float* cs, int* cr, uint32_t* cx, int k, float* out_s, int64_t* out_r,
                       int force, hipStream_t st);
constexpr bool screen_valu_inline_fallback(int nqt, int dtype, int D) {
  return nqt == 1 && !(dtype == RFX_F32 && D == 1024);  // (f32 at d 1024: the two bodies together spill)
}

// ---- MFMA scan (batched bf16 / f16) -------------------------------------------------------
struct MfmaPlan {
  int bn;          // queries per workgroup tile (64/128/256)
  int q_blocks;    // gridDim.y
  int k_lane;      // lane-list length (>= k)
  int blocks;      // gridDim.x (persistent over row tiles)
  int tiles_per_block;
  int lists_per_block;  // lane lists per query per block
  int64_t n_lists;      // per query
  int64_t nq_pad;
  bool ok;
};
MfmaPlan plan_scan_mfma(int64_t nrows, int D, int dtype, int64_t nq, int k);
int launch_scan_mfma(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad,
                     int nq, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr);
int launch_scan_mfma_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int D, const void* Qpad, int nq,
                         float* cs, int* cr, hipStream_t st);
MfmaPlan plan_scan_mfma2(int64_t nrows, int D, int dtype, int64_t nq, int k);
int launch_scan_mfma2(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr);
int launch_scan_mfma2_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int D, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st);
MfmaPlan plan_scan_mfma3(int64_t nrows, int D, int dtype, int64_t nq, int k);
int launch_scan_mfma3(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr);
size_t tau_bytes_mfma6(const MfmaPlan& p);
MfmaPlan plan_scan_mfma6(int64_t nrows, int D, int dtype, int64_t nq, int k);
// gate (optional): a device word; the launch does nothing unless it is non-zero (the exact pass of
// the two-pass scan runs only when the screen's select kernel asked for it)
int launch_scan_mfma6(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr,
                      const uint32_t* gate = nullptr, bool tau_zeroed = false);
int launch_scan_mfma6_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int dtype, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st);
size_t tau_bytes_mfma8(const MfmaPlan& p);
MfmaPlan plan_scan_mfma8(int64_t nrows, int D, int dtype, int64_t nq, int k);
int launch_scan_mfma8(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr,
                      const uint32_t* gate = nullptr, bool tau_zeroed = false);
// f32 stores (kernel 9): batched scan on v_mfma_f32_16x16x4_f32 for 16 < nq
size_t tau_bytes_mfma9(const MfmaPlan& p);
MfmaPlan plan_scan_mfma9(int64_t nrows, int D, int dtype, int64_t nq, int k);
// gate / tau_zeroed: as kernel 6 (the exact pass of the two-pass scan of an f32 store)
int launch_scan_mfma9(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask = nullptr,
                      const uint32_t* gate = nullptr, bool tau_zeroed = false);
void launch_pad_queries(const void* Q, int64_t nq, int64_t nq_pad, int D, int esz, void* out,
                        hipStream_t st);

// ---- merge -----------------------------------------------------------------------------------
int launch_topk_merge(const float* cs, const void* cr, int rows_are_i64, int64_t nq, int64_t n_cand,
                      int k, int64_t row_offset, float* out_s, int64_t* out_r, hipStream_t st);
int launch_topk_merge_lists(const float* cs, const void* cr, int rows_are_i64, int64_t nq, int64_t n_cand,
                            int list_len, int k, int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec,
                            hipStream_t st,
                            bool sorted = false, const uint32_t* gate = nullptr, const Rescore* rescore = nullptr);
int launch_merge_gathered(const void* rec, int world, int64_t nq, int k, float* out_s, int64_t* out_r,
                          hipStream_t st);
// n (score, row) pairs -> {score, 0, row + row_offset} merge records (rec) or (out_s, out_r + row_offset);
// padding rows (< 0) stay -1
void launch_rescore_topk(const Rescore& rs, int64_t nq, int k, int64_t row_offset, float* out_s, int64_t* out_r,
                         void* out_rec, hipStream_t st);
void launch_pack_records(const float* s, const int64_t* r, int64_t n, int64_t row_offset, void* rec, float* out_s,
                         int64_t* out_r, hipStream_t st);

// ---- the exact two-pass scan (kernel 10 + k_screen.hip) -----------------------------
bool screen_supported(int D, int dtype);
// int8 copy of tiles [tile0, tile0 + ntiles) (tiles_d == nullptr) or of the ntiles tiles listed in tiles_d
// tmeta: per tile 16 B {f32 scale, u32 live word, 0, 0}
void launch_screen_quantize(const void* X, int D, int dtype, int64_t tile0, int64_t ntiles, const int64_t* tiles_d,
                            int8_t* codes, void* tmeta, uint32_t* stats, hipStream_t st);
MfmaPlan plan_scan_screen(int64_t nrows, int D, int dtype, int64_t nq, int k, int max_blocks = 0);
size_t tau_bytes_screen(const MfmaPlan& p);
uint32_t* xcd_weights_device_ptr();  // kernel 10's per-device XCD weight table (k_screen.hip g_xcd_w)
// ftau (or null): the gated fallback scan's threshold table ([nq_pad][kFallbackTauW], kernel 6 / 8),
// zeroed here so the fallback launch needs no memset of its own (tau_zeroed below)
constexpr int kFallbackTauW = 16;
// ftau_nq: the fallback's padded batch (its table rows zeroed; may exceed nq_pad).  sd (kernel 10's plans):
// the int8 copy, its rows, the row mask and the lane-list length, from which each query's seed bound is taken
// (k_screen.hip); nullptr: the seed words are zeroed (no seed)
struct ScreenSeed {
  const int8_t* X8 = nullptr;
  const void* tmeta = nullptr;
  int nrows = 0;
  const uint32_t* mask = nullptr;
  int kl = 0;
};
void launch_screen_queries(const void* Q, int dtype, int D, int64_t nq, int64_t nq_pad, int8_t* Qc, float* qe2,
                           const uint32_t* stats, uint32_t* tau, uint32_t* gate, uint32_t* ftau, int64_t ftau_nq,
                           hipStream_t st, const ScreenSeed* sd = nullptr);
int launch_scan_screen(const MfmaPlan& p, const int8_t* codes, const void* tmeta, const uint32_t* stats, int nrows, int D,
                       const int8_t* Qc, const float* qe2, int nq, uint32_t* tau, float* cs, int* cr, uint32_t* drops,
                       hipStream_t st, const uint32_t* mask);
int launch_screen_select(const float* cs, const int* cr, const uint32_t* drops, int64_t n_lists, int list_len,
                         const float* qe2, const void* Q, const void* X, int D, int dtype, int64_t nq, int k,
                         int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec, uint32_t* gate, int* diag,
                         int force, hipStream_t st);

// ---- embedding ---------------------------------------------------------------------------------
void launch_embed_weights(int V, int dim, uint64_t seed, void* wt, hipStream_t st);
int launch_embed(const int32_t* indptr, const int32_t* bucket, const int16_t* count, int64_t n, int V,
                 const void* wt, int dim, void* out, int out_dtype, void* ws, hipStream_t st);

// ---- IVF-Flat int8 (k_ivf.hip) --------------------------------------------------------------------
namespace ivf {
void launch_synth_clustered(uint64_t cseed, uint64_t ncenters, uint64_t seed, int64_t row0, int64_t n, int dim,
                            int dtype, void* out, hipStream_t st);
void launch_quantize(const void* X, int64_t n, int dim, int dtype, int8_t* codes, float* inv, hipStream_t st);
int launch_coarse_scores(const int8_t* X, int64_t n, const int8_t* C, int m, int D, const float* fc, float* S,
                         int* ids, hipStream_t st);
int launch_assign(const int8_t* X, int64_t n, const int8_t* C, int m, int D, const float* fc, int* labels,
                  float* best, hipStream_t st);
void launch_init_centroids(const int8_t* codes, int64_t step, int m, int D, int8_t* qc, hipStream_t st);
void launch_kmeans_accum(const int8_t* X, int64_t n, int D, const int* labels, int* sums, int* counts,
                         hipStream_t st);
// sums == nullptr: only recompute the factors of qc
void launch_centroid_update(const int* sums, const int* counts, int m, int D, int8_t* qc, float* fc, hipStream_t st);
size_t sort_temp_bytes(int64_t n);
int launch_build_lists(const int* labels, int64_t n, int m, const int8_t* codes, const float* inv, int D,
                       unsigned* keys_tmp, int* vals_tmp, unsigned* keys_out, int* ids_out, void* sort_tmp,
                       size_t sort_tmp_bytes, int* counts, int64_t* off, int8_t* dcodes, float* dinv,
                       hipStream_t st);
int list_k(int k);
// each query's nprobe best of m coarse scores (m <= 4096; else -1: use launch_topk_merge), in no order
int launch_probe_select(const float* S, int64_t nq, int m, int nprobe, float* ps, int64_t* pid, hipStream_t st);
int launch_group_pairs(const int64_t* probes, int P, int m, int* pair_off, int* pairs, hipStream_t st);
int launch_list_scan(int K, int D, int m, int splits, const int8_t* codes, const float* inv, const int* ids, const int64_t* off,
                     const int* pair_off, const int* pairs, int nprobe, const int8_t* qq, const float* qinv,
                     float* cs, int* cr, hipStream_t st);
int launch_rerank(const void* Q, int dtq, const void* X, int dtx, int D, const int64_t* cand, int64_t nq, int kc,
                  float* out_s, int64_t* out_r, hipStream_t st, int64_t row_lo = 0, int64_t n_rows = INT64_MAX);
}  // namespace ivf

// error reporting shared by the C-ABI translation units (rfx_api.hip owns rfx_last_error)
int api_fail(int code, const char* fmt, ...);

}  // namespace rfx
