// k_embed.hip — chunk embedding as a dense MFMA contraction (index write of upload_file,
// backend/app/services/gemini_rag.py:319-327, whose embedding the reference leaves to Gemini).
//
//   F  [n][V]   bf16  signed hashed token counts of each chunk (|count| <= 256: exact in bf16)
//   WT [dim][V] bf16  seeded projection, entries w/128 with w in [-127,127] (exact in bf16)
//   E = F · W   f32   every partial sum is an integer multiple of 2^-7 below 2^17 in magnitude
//                     (chunks are capped at 65536 tokens), so the f32 MFMA accumulation is EXACT
//                     in any order -> embeddings are bit-identical to oracle/embed.py.
//   x = e / sqrt(sum e^2) with the sum in int64 and the scale in f64, rounded to f32, then to
//   the index dtype (same rule as the synthetic generator).
// MFMA tile: one 256-thread workgroup = 32 chunk rows × all dim columns; wave w owns 32-col
// sub-tiles w, w+4, ... (v_mfma_f32_32x32x16_bf16).  Operands stream straight to VGPRs
// (WT is re-read from L2/MALL by every workgroup; F rows are read once).
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {

typedef __attribute__((ext_vector_type(8))) __bf16 ebf16x8_t;
typedef __attribute__((ext_vector_type(16))) float ef32x16_t;

// ---- projection weights --------------------------------------------------------------------
__global__ void embed_weights_kernel(uint64_t base, int V, int dim, uint16_t* __restrict__ wt) {
  const int64_t total = (int64_t)V * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t u = splitmix64(base + (uint64_t)i);
    const int w = (int)(((u >> 32) * 255ull) >> 32) - 127;  // uniform in [-127, 127]
    wt[i] = f32_to_bf16((float)w * (1.0f / 128.0f));
  }
}

void launch_embed_weights(int V, int dim, uint64_t seed, void* wt, hipStream_t st) {
  const int64_t total = (int64_t)V * dim;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(embed_weights_kernel, dim3(blocks), dim3(256), 0, st, splitmix64(seed), V, dim,
                     (uint16_t*)wt);
}

// ---- CSR -> dense bf16 features ---------------------------------------------------------------
__global__ void densify_kernel(const int32_t* __restrict__ indptr, const int32_t* __restrict__ bucket,
                               const int16_t* __restrict__ count, int V, uint16_t* __restrict__ F) {
  const int64_t c = blockIdx.x;
  const int b = indptr[c], e = indptr[c + 1];
  for (int i = b + threadIdx.x; i < e; i += blockDim.x)
    F[c * V + bucket[i]] = f32_to_bf16((float)count[i]);
}

// ---- GEMM + exact normalisation ----------------------------------------------------------------
template <int NSUB, int ODT>
__global__ __launch_bounds__(256) void embed_gemm_kernel(const uint16_t* __restrict__ F, int64_t n, int V,
                                                         const uint16_t* __restrict__ WT, int dim,
                                                         void* __restrict__ out) {
  __shared__ long long ss_part[4][32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t row0 = (int64_t)blockIdx.x * 32;
  const int nsub_total = dim / 32;

  ef32x16_t acc[NSUB];
#pragma unroll
  for (int s = 0; s < NSUB; ++s)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[s][r] = 0.f;

  const int64_t arow = row0 + l32;
  const uint16_t* fa = F + (arow < n ? arow : 0) * (int64_t)V + 8 * half;
  for (int k0 = 0; k0 < V; k0 += 16) {
    uint4 a = arow < n ? *(const uint4*)(fa + k0) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
      const int sub = w + 4 * s;
      if (sub < nsub_total) {
        const uint4 b = *(const uint4*)(WT + (int64_t)(sub * 32 + l32) * V + k0 + 8 * half);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(ebf16x8_t, a),
                                                         __builtin_bit_cast(ebf16x8_t, b), acc[s], 0, 0, 0);
      }
    }
  }

  // exact integer view: e = E * 128 (|e| < 2^24)
  long long part[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) part[r] = 0;
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    if (w + 4 * s < nsub_total) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long e = (long long)(acc[s][r] * 128.0f);
        part[r] += e * e;
      }
    }
  }
  // reduce over the 32 lanes that share rows (same half), then over the 4 waves
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int off = 16; off; off >>= 1) part[r] += __shfl_xor(part[r], off);
  }
  if (l32 == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ss_part[w][(r & 3) + 8 * (r >> 2) + 4 * half] = part[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = (r & 3) + 8 * (r >> 2) + 4 * half;
    const int64_t row = row0 + rr;
    if (row >= n) continue;
    const long long S = ss_part[0][rr] + ss_part[1][rr] + ss_part[2][rr] + ss_part[3][rr];
    const double scale = S > 0 ? 1.0 / sqrt((double)S) : 0.0;
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
      const int sub = w + 4 * s;
      if (sub >= nsub_total) continue;
      const int col = sub * 32 + l32;
      const long long e = (long long)(acc[s][r] * 128.0f);
      const float x = (float)((double)e * scale);
      if constexpr (ODT == RFX_F32)
        ((float*)out)[row * dim + col] = x;
      else if constexpr (ODT == RFX_BF16)
        ((uint16_t*)out)[row * dim + col] = f32_to_bf16(x);
      else
        ((uint16_t*)out)[row * dim + col] = f32_to_f16(x);
    }
  }
}

template <int NSUB>
static void launch_gemm_odt(int odt, dim3 grid, hipStream_t st, const uint16_t* F, int64_t n, int V,
                            const uint16_t* WT, int dim, void* out) {
  if (odt == RFX_F32)
    hipLaunchKernelGGL((embed_gemm_kernel<NSUB, RFX_F32>), grid, dim3(256), 0, st, F, n, V, WT, dim, out);
  else if (odt == RFX_BF16)
    hipLaunchKernelGGL((embed_gemm_kernel<NSUB, RFX_BF16>), grid, dim3(256), 0, st, F, n, V, WT, dim, out);
  else
    hipLaunchKernelGGL((embed_gemm_kernel<NSUB, RFX_F16>), grid, dim3(256), 0, st, F, n, V, WT, dim, out);
}

// ws: dense F [n][V] bf16 (n*V*2 bytes)
int launch_embed(const int32_t* indptr, const int32_t* bucket, const int16_t* count, int64_t n, int V,
                 const void* wt, int dim, void* out, int out_dtype, void* ws, hipStream_t st) {
  if (n <= 0) return 0;
  uint16_t* F = (uint16_t*)ws;
  if (hipMemsetAsync(F, 0, (size_t)n * V * 2, st) != hipSuccess) return -2;
  hipLaunchKernelGGL(densify_kernel, dim3((unsigned)n), dim3(256), 0, st, indptr, bucket, count, V, F);
  const int nsub = (dim / 32 + 3) / 4;
  dim3 grid((unsigned)((n + 31) / 32));
  const uint16_t* WT = (const uint16_t*)wt;
  if (nsub <= 2)
    launch_gemm_odt<2>(out_dtype, grid, st, F, n, V, WT, dim, out);
  else if (nsub <= 4)
    launch_gemm_odt<4>(out_dtype, grid, st, F, n, V, WT, dim, out);
  else if (nsub <= 6)
    launch_gemm_odt<6>(out_dtype, grid, st, F, n, V, WT, dim, out);
  else if (nsub <= 8)
    launch_gemm_odt<8>(out_dtype, grid, st, F, n, V, WT, dim, out);
  else
    return -1;
  return 0;
}

}  // namespace rfx
