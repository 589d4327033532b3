// k_scan_valu.hip — synthetic row generator, the VALU scan's plan and launchers (kernel template:
// k_scan_valu.h, instantiated in valu_<dtype>.hip), query widening, and the top-k merge kernels.
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
#include "k_scan_valu.h"

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
  if (dtype == RFX_F32) return launch_valu_f32(p, X, nrows, D, Qf, nq, cs, cr, st, mask, tau, fo);
  if (dtype == RFX_BF16) return launch_valu_bf16(p, X, nrows, D, Qf, nq, cs, cr, st, mask, tau, fo);
  return launch_valu_f16(p, X, nrows, D, Qf, nq, cs, cr, st, mask, tau, fo);
}

int launch_scan_valu(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const float* Qf, int nq,
                     float* cs, int* cr, hipStream_t st, const uint32_t* mask, uint32_t* tau) {
  return launch_valu(p, X, nrows, D, dtype, Qf, nq, cs, cr, st, mask, tau, FusedOut{nullptr, 0, nullptr, nullptr});
}

int launch_search_valu_fused(const ValuPlan& p, const void* X, int nrows, int D, int dtype, const void* Q, int nq,
                             float* cs, int* cr, uint32_t* state, int k, float* out_s, int64_t* out_r,
                             hipStream_t st, const uint32_t* mask, const uint32_t* gate) {
  // state: [kFusedMaxNq] bounds then [q_slices] counters, all zero (and left zero)
  return launch_valu(p, X, nrows, D, dtype, Q, nq, cs, cr, st, mask, state,
                     FusedOut{state + kValuFusedMaxNq, k, out_s, out_r, gate});
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

template <int K, bool R64, bool SORTED, class Src>
__global__ __launch_bounds__(512) void merge_kernel(Src src, int list_len, int k_out, int64_t row_offset,
                                                    float* __restrict__ out_s, int64_t* __restrict__ out_r,
                                                    MergeRec* __restrict__ out_rec, const uint32_t* __restrict__ gate,
                                                    Rescore rs) {
  if (gate && *gate == 0u) return;  // the two-pass scan's gated fallback (k_screen.hip)
  merge_one<K, R64, 8, SORTED>(src, (int64_t)blockIdx.x, list_len, k_out, row_offset, out_s, out_r, out_rec);
  if (rs.X) rescore_final(rs, (int64_t)blockIdx.x, k_out, row_offset, out_s, out_r, out_rec);
}

// The score rule applied to an answer in place (rfx_rescore_topk): one 256-thread block per query re-scores
// its k entries (fl32 of the f64 dot with the index rows) and re-orders them (score desc, row asc).
__global__ __launch_bounds__(256) void rescore_topk_kernel(Rescore rs, int k, int64_t row_offset, float* __restrict__ out_s,
                                                           int64_t* __restrict__ out_r, MergeRec* __restrict__ out_rec) {
  rescore_final(rs, (int64_t)blockIdx.x, k, row_offset, out_s, out_r, out_rec);
}

void launch_rescore_topk(const Rescore& rs, int64_t nq, int k, int64_t row_offset, float* out_s, int64_t* out_r,
                         void* out_rec, hipStream_t st) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(rescore_topk_kernel, dim3((unsigned)nq), dim3(256), 0, st, rs, k, row_offset, out_s, out_r,
                     (MergeRec*)out_rec);
}

int launch_topk_merge_lists(const float* cs, const void* cr, int rows_are_i64, int64_t nq, int64_t n_cand,
                            int list_len, int k, int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec,
                            hipStream_t st, bool sorted, const uint32_t* gate, const Rescore* rescore) {
  const Rescore rs = rescore ? *rescore : Rescore{};
  const int kk = valu_k_slot(k);
  if (nq <= 0) return 0;
  if (list_len < 1 || (list_len > 1 && n_cand % list_len != 0)) {
    list_len = 1;
    sorted = false;
  }
  MergeRec* rec = (MergeRec*)out_rec;
#define RFX_M2(KV, R, S)                                                                                  \
  hipLaunchKernelGGL((merge_kernel<KV, R, S, FlatSrc<R>>), dim3((unsigned)nq), dim3(512), 0, st,          \
                     FlatSrc<R>{cs, cr, n_cand}, list_len, k, row_offset, out_s, out_r, rec, gate, rs)
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

// The gathered merge of the multi-GPU step: `world` sorted lists of k records per query (every rank's
// top-k, best first, padding (-inf, -1) at the tail).  One wave per query, 4 queries per block: the
// world * k records are staged in LDS and every live record finds its final rank as its index in
// its own list plus, for each other list, the number of records better than it (binary search,
// broadcast LDS reads): world * log2(k) reads per record, no serial chain, no block-wide list
// (config 3 at 8 GPUs: 80 records per query, 64 blocks).  Ranks of distinct (score, row) pairs are
// distinct, so each of the k best lands in its own slot; slots past the live count get padding.
constexpr int kGatherSmallMax = 512;  // world * k staged per wave; larger gathers take merge_kernel

__global__ __launch_bounds__(256) void merge_gathered_small_kernel(const MergeRec* __restrict__ rec, int world,
                                                                   int64_t nq, int k, float* __restrict__ out_s,
                                                                   int64_t* __restrict__ out_r) {
  __shared__ float ss[4][kGatherSmallMax];
  __shared__ long long sr[4][kGatherSmallMax];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  const bool active = q < nq;
  const int n = world * k;
  int live_n = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    bool live = false;
    if (active && i < n) {
      const int m = i / k, e = i - m * k;
      const MergeRec r = rec[((int64_t)m * nq + q) * k + e];
      live = r.r >= 0 && r.r != kNoRow && r.s == r.s;
      ss[w][i] = r.s;
      sr[w][i] = live ? r.r : kNoRow;
    }
    live_n += __popcll(__ballot(live));
  }
  __syncthreads();
  if (!active) return;
  for (int i = lane; i < n; i += 64) {
    const long long r = sr[w][i];
    if (r == kNoRow) continue;
    const float s = ss[w][i];
    const int m = i / k;
    int rank = i - m * k;
    for (int mm = 0; mm < world && rank < k; ++mm) {
      if (mm == m) continue;
      const float* ls = ss[w] + mm * k;
      const long long* lr = sr[w] + mm * k;
      int lo = 0, hi = k;  // first record of list mm that is not better than (s, r)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (lr[mid] != kNoRow && better64(ls[mid], lr[mid], s, r))
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      out_s[q * k + rank] = s;
      out_r[q * k + rank] = r;
    }
  }
  for (int i = live_n + lane; i < k; i += 64) {
    out_s[q * k + i] = -__builtin_inff();
    out_r[q * k + i] = -1;
  }
}

int launch_merge_gathered(const void* rec, int world, int64_t nq, int k, float* out_s, int64_t* out_r,
                          hipStream_t st) {
  const int kk = valu_k_slot(k);
  if (nq <= 0) return 0;
  if ((int64_t)world * k <= kGatherSmallMax) {
    hipLaunchKernelGGL(merge_gathered_small_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, st,
                       (const MergeRec*)rec, world, nq, k, out_s, out_r);
    return 0;
  }
  GatheredSrc src{(const MergeRec*)rec, nq, k, (int64_t)world * k};
#define RFX_M(KV)                                                                                     \
  if (kk == KV) {                                                                                     \
    hipLaunchKernelGGL((merge_kernel<KV, true, true, GatheredSrc>), dim3((unsigned)nq), dim3(512), 0, st, \
                       src, k, k, 0, out_s, out_r, nullptr, nullptr, Rescore{});                               \
    return 0;                                                                                         \
  }
  RFX_VALU_K_LIST(RFX_M)
#undef RFX_M
  return -1;
}

__global__ __launch_bounds__(256) void pack_records_kernel(const float* __restrict__ s, const int64_t* __restrict__ r,
                                                           int64_t n, int64_t row_offset, MergeRec* __restrict__ rec,
                                                           float* __restrict__ out_s, int64_t* __restrict__ out_r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float sc = s[i];
  const int64_t rr = r[i];
  const int64_t g = rr < 0 ? -1 : rr + row_offset;
  if (rec) {
    rec[i] = MergeRec{sc, 0, (long long)g};
  } else {
    out_s[i] = sc;
    out_r[i] = g;
  }
}

void launch_pack_records(const float* s, const int64_t* r, int64_t n, int64_t row_offset, void* rec, float* out_s,
                         int64_t* out_r, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(pack_records_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, r, n, row_offset,
                     (MergeRec*)rec, out_s, out_r);
}

}  // namespace rfx
