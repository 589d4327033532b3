// k_ivf.hip — IVF-Flat int8 (build plan item 8): clustered synthetic rows,
// int8 quantisation, MFMA i8 coarse scoring (k-means assignment and probe selection), k-means
// update, posting-list build and the posting-list scan.
//
// Numerics are exact by construction (oracle/ivf.py restates them and the GPU is held to it
// bit-for-bit): int8 x int8 dot products accumulate in int32 (|dot| <= 768·127² < 2^24, so the
// f32 conversion is exact too), and every floating-point step is ONE correctly rounded IEEE op
// (__fdiv_rn / __fmul_rn / __fsqrt_rn, rintf) that numpy's float32 performs identically.
#include <rocprim/device/device_radix_sort.hpp>

#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {
namespace ivf {

typedef __attribute__((ext_vector_type(4))) int v4i;
typedef __attribute__((ext_vector_type(16))) int v16i;

constexpr uint64_t kCentreKey = 1ull << 63;  // generator key spaces (oracle/ivf.py C_KEY, L_KEY)
constexpr uint64_t kLabelKey = 1ull << 62;

// ---- clustered synthetic rows: centre(cluster(r)) + noise(r), normalised exactly ---------------
template <int DT>
__global__ __launch_bounds__(256) void synth_clustered_kernel(uint64_t bc, uint64_t bn, uint64_t ncenters,
                                                              int64_t row0, int64_t n, int dim,
                                                              void* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nwaves) {
    const uint64_t r = (uint64_t)(row0 + i);
    const uint64_t lab = (splitmix64(bn + kLabelKey + r) >> 32) % ncenters;
    const uint64_t ck = kCentreKey + lab * (uint64_t)dim, nk = r * (uint64_t)dim;
    long long ss = 0;
    for (int c = lane; c < dim; c += 64) {
      const long long v = (long long)synth_raw(bc, ck + c) + synth_raw(bn, nk + c);
      ss += v * v;
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) ss += __shfl_xor(ss, off);
    const double rs = ss > 0 ? 1.0 / sqrt((double)ss) : 0.0;
    for (int c = lane; c < dim; c += 64) {
      const long long v = (long long)synth_raw(bc, ck + c) + synth_raw(bn, nk + c);
      const float x = (float)((double)v * rs);
      if constexpr (DT == RFX_F32)
        ((float*)out)[i * dim + c] = x;
      else if constexpr (DT == RFX_BF16)
        ((uint16_t*)out)[i * dim + c] = f32_to_bf16(x);
      else
        ((uint16_t*)out)[i * dim + c] = f32_to_f16(x);
    }
  }
}

void launch_synth_clustered(uint64_t cseed, uint64_t ncenters, uint64_t seed, int64_t row0, int64_t n, int dim,
                            int dtype, void* out, hipStream_t st) {
  const uint64_t bc = splitmix64(cseed), bn = splitmix64(seed);
  const int blocks = (int)std::min<int64_t>((std::max<int64_t>(n, 1) + 3) / 4, 8192);
  if (dtype == RFX_F32)
    hipLaunchKernelGGL(synth_clustered_kernel<RFX_F32>, dim3(blocks), dim3(256), 0, st, bc, bn, ncenters, row0, n, dim, out);
  else if (dtype == RFX_BF16)
    hipLaunchKernelGGL(synth_clustered_kernel<RFX_BF16>, dim3(blocks), dim3(256), 0, st, bc, bn, ncenters, row0, n, dim, out);
  else
    hipLaunchKernelGGL(synth_clustered_kernel<RFX_F16>, dim3(blocks), dim3(256), 0, st, bc, bn, ncenters, row0, n, dim, out);
}

// ---- int8 quantisation (one wave per row) --------------------------------------------------------
template <int DT>
__device__ __forceinline__ float load_elem(const void* X, int64_t i) {
  if constexpr (DT == RFX_F32)
    return ((const float*)X)[i];
  else if constexpr (DT == RFX_BF16)
    return bf16_to_f32(((const uint16_t*)X)[i]);
  else
    return f16_to_f32(((const uint16_t*)X)[i]);
}

template <int DT>
__global__ __launch_bounds__(256) void quantize_kernel(const void* __restrict__ X, int64_t n, int dim,
                                                       int8_t* __restrict__ codes, float* __restrict__ inv) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nwaves) {
    float amax = 0.f;
    for (int c = lane; c < dim; c += 64) amax = fmaxf(amax, fabsf(load_elem<DT>(X, i * dim + c)));
#pragma unroll
    for (int off = 32; off; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    const float s = amax > 0.f ? __fdiv_rn(127.f, amax) : 0.f;
    for (int c = lane; c < dim; c += 64) {
      const float q = rintf(__fmul_rn(load_elem<DT>(X, i * dim + c), s));
      codes[i * dim + c] = (int8_t)fminf(fmaxf(q, -127.f), 127.f);
    }
    if (lane == 0) inv[i] = __fdiv_rn(amax, 127.f);
  }
}

void launch_quantize(const void* X, int64_t n, int dim, int dtype, int8_t* codes, float* inv, hipStream_t st) {
  const int blocks = (int)std::min<int64_t>((std::max<int64_t>(n, 1) + 3) / 4, 8192);
  if (dtype == RFX_F32)
    hipLaunchKernelGGL(quantize_kernel<RFX_F32>, dim3(blocks), dim3(256), 0, st, X, n, dim, codes, inv);
  else if (dtype == RFX_BF16)
    hipLaunchKernelGGL(quantize_kernel<RFX_BF16>, dim3(blocks), dim3(256), 0, st, X, n, dim, codes, inv);
  else
    hipLaunchKernelGGL(quantize_kernel<RFX_F16>, dim3(blocks), dim3(256), 0, st, X, n, dim, codes, inv);
}

// ---- coarse scoring: MFMA i8 (v_mfma_i32_32x32x32_i8) -------------------------------------------
// Block: 128 rows of X (queries / rows to assign) resident in LDS, the centroid table streamed in
// 128-centroid × 64-byte chunks (double-buffered).  4 waves in a 2×2 grid, each 64 centroids ×
// 64 X rows = 2×2 MFMA tiles.  A operand = centroids (accumulator rows), B = X rows (accumulator
// columns = lanes), so a lane holds 16 centroids of ONE X row: the argmax is in-lane.
// LDS images are XOR-swizzled by 16-byte chunk: X row r chunk c at c ^ (r & xs_mask); centroid
// row r (64 B) chunk c at c ^ ((r >> 2) & 3): the 32-row fragment reads hit distinct banks.
constexpr int kXT = 128, kCT = 128, kKC = 64, kMaxD = 1024;
constexpr int kXBytes = kXT * kMaxD, kCBytes = kCT * kKC;

__device__ __forceinline__ v16i mfma_i8(const uint4& a, const uint4& b, const v16i& c) {
  v4i av = {(int)a.x, (int)a.y, (int)a.z, (int)a.w}, bv = {(int)b.x, (int)b.y, (int)b.z, (int)b.w};
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
}

// MODE 0: write scores S[x][c] = f32(dot) * fc[c] and ids[x][c] = c (probe selection: the merge
// kernel then takes the top nprobe per row); grid.y splits the centroids.
// MODE 1: labels[x] = argmax_c (f32(dot) * fc[c]), ties -> lowest c (k-means / list assignment).
template <int MODE>
__global__ __launch_bounds__(256, 1) void coarse_kernel(const int8_t* __restrict__ X, int64_t n,
                                                        const int8_t* __restrict__ C, int m, int D,
                                                        const float* __restrict__ fc, int ctiles_per_block,
                                                        float* __restrict__ out_s, int* __restrict__ out_i) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kXBytes + 2 * kCBytes];
  uint8_t* const xs = lds;
  uint8_t* const cs = lds + kXBytes;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm = w & 1, wn = w >> 1;
  const int64_t x0 = (int64_t)blockIdx.x * kXT;
  const int nch = D >> 4;  // 16-byte chunks per X row
  const int xs_mask = min(15, (nch & -nch) - 1);
  const int ctiles = (m + kCT - 1) / kCT;
  const int ct0 = blockIdx.y * ctiles_per_block;
  const int ct1 = min(ctiles, ct0 + ctiles_per_block);
  const int nk = D / kKC;
  const int T = (ct1 - ct0) * nk;
  if (T <= 0) return;

  // resident X tile
  for (int i = tid; i < kXT * nch; i += 256) {
    const int r = i / nch, c = i - r * nch;
    const int64_t xr = min(x0 + r, n - 1);
    const uint4 v = *(const uint4*)(X + xr * D + c * 16);
    *(uint4*)(xs + r * D + (((c & ~xs_mask) | ((c ^ r) & xs_mask)) << 4)) = v;
  }
  auto load_c = [&](int t, uint4 (&v)[2]) {
    const int ct = ct0 + t / nk, kc = t - (t / nk) * nk;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u, r = i >> 2, c = i & 3;
      const int cr = ct * kCT + r;
      v[u] = cr < m ? *(const uint4*)(C + (int64_t)cr * D + kc * kKC + c * 16) : uint4{0u, 0u, 0u, 0u};
    }
  };
  auto store_c = [&](int buf, const uint4 (&v)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u, r = i >> 2, c = i & 3;
      *(uint4*)(cs + buf * kCBytes + r * kKC + ((c ^ ((r >> 2) & 3)) << 4)) = v[u];
    }
  };
  {
    uint4 v[2];
    load_c(0, v);
    store_c(0, v);
  }
  __syncthreads();

  v16i acc[2][2];
  float bs[2] = {-__builtin_inff(), -__builtin_inff()};
  int bc[2] = {0x7fffffff, 0x7fffffff};
  for (int t = 0; t < T; ++t) {
    const int kc = t % nk;
    if (kc == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = v16i{};
    }
    uint4 nv[2];
    if (t + 1 < T) load_c(t + 1, nv);
    const uint8_t* cb = cs + (t & 1) * kCBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // two 32-deep k-steps per 64-byte chunk
      const int cc = 2 * s + h;
      uint4 a[2], b[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int r = wm * 64 + mi * 32 + l32;
        a[mi] = *(const uint4*)(cb + r * kKC + ((cc ^ ((r >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int r = wn * 64 + ni * 32 + l32;
        const int c = kc * 4 + cc;
        b[ni] = *(const uint4*)(xs + r * D + (((c & ~xs_mask) | ((c ^ r) & xs_mask)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          // MODE 0: X rows as accumulator rows, centroids as lanes, so the score rows go out in 128-B runs
          if constexpr (MODE == 0)
            acc[mi][ni] = mfma_i8(b[ni], a[mi], acc[mi][ni]);
          else
            acc[mi][ni] = mfma_i8(a[mi], b[ni], acc[mi][ni]);
        }
    }
    if (t + 1 < T) store_c((t + 1) & 1, nv);
    if (MODE == 0 && kc == nk - 1) {
      // round 6: lane l32 holds centroid cbase + 32 mi + l32 for 16 X rows, so each store of a row's scores
      // is 32 consecutive floats (before: a lane per X row, 16-KB strides between lanes; 43.7 us per batch)
      const int cbase = (ct0 + t / nk) * kCT + wm * 64;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int c = cbase + mi * 32 + l32;
        const bool cok = c < m;
        const float fcc = cok ? fc[c] : 0.f;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t x = x0 + wn * 64 + ni * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (cok && x < n) {
              out_s[x * m + c] = __fmul_rn((float)acc[mi][ni][r], fcc);
              out_i[x * m + c] = c;
            }
          }
      }
    }
    if (MODE == 1 && kc == nk - 1) {
      const int cbase = (ct0 + t / nk) * kCT + wm * 64;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int64_t x = x0 + wn * 64 + ni * 32 + l32;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = cbase + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (c < m) {
              const float f = __fmul_rn((float)acc[mi][ni][r], fc[c]);
              if (f > bs[ni] || (f == bs[ni] && c < bc[ni])) {
                bs[ni] = f;
                bc[ni] = c;
              }
            }
          }
      }
    }
    __syncthreads();
  }
  if constexpr (MODE == 1) {
    // combine the two lane halves (disjoint centroid rows), then the two centroid-half waves
    float* rs = (float*)cs;      // [2 wn][64] scores
    int* ri = (int*)(cs + 512);  // [2 wn][64] ids
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const float os = __shfl_xor(bs[ni], 32);
      const int oc = __shfl_xor(bc[ni], 32);
      if (os > bs[ni] || (os == bs[ni] && oc < bc[ni])) {
        bs[ni] = os;
        bc[ni] = oc;
      }
      if (wm == 1 && h == 0) {
        rs[wn * 64 + ni * 32 + l32] = bs[ni];
        ri[wn * 64 + ni * 32 + l32] = bc[ni];
      }
    }
    __syncthreads();
    if (wm == 0 && h == 0) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const float os = rs[wn * 64 + ni * 32 + l32];
        const int oc = ri[wn * 64 + ni * 32 + l32];
        if (os > bs[ni] || (os == bs[ni] && oc < bc[ni])) {
          bs[ni] = os;
          bc[ni] = oc;
        }
        const int64_t x = x0 + wn * 64 + ni * 32 + l32;
        if (x < n) {
          out_i[x] = bc[ni];
          if (out_s) out_s[x] = bs[ni];
        }
      }
    }
  }
}

int launch_coarse_scores(const int8_t* X, int64_t n, const int8_t* C, int m, int D, const float* fc, float* S,
                         int* ids, hipStream_t st) {
  if (D % kKC || D > kMaxD || n <= 0 || m <= 0) return -1;
  const int64_t xb = (n + kXT - 1) / kXT;
  const int ctiles = (m + kCT - 1) / kCT;
  // spread the (few) query tiles over the chip: ~512 blocks
  const int splits = (int)std::max<int64_t>(1, std::min<int64_t>(ctiles, 512 / std::max<int64_t>(xb, 1)));
  const int per = (ctiles + splits - 1) / splits;
  dim3 grid((unsigned)xb, (unsigned)((ctiles + per - 1) / per));
  hipLaunchKernelGGL(coarse_kernel<0>, grid, dim3(256), 0, st, X, n, C, m, D, fc, per, S, ids);
  return 0;
}

int launch_assign(const int8_t* X, int64_t n, const int8_t* C, int m, int D, const float* fc, int* labels,
                  float* best, hipStream_t st) {
  if (D % kKC || D > kMaxD || n <= 0 || m <= 0) return -1;
  const int64_t xb = (n + kXT - 1) / kXT;
  if (xb > 0x7fffffff) return -1;
  const int ctiles = (m + kCT - 1) / kCT;
  hipLaunchKernelGGL(coarse_kernel<1>, dim3((unsigned)xb, 1), dim3(256), 0, st, X, n, C, m, D, fc, ctiles, best,
                     labels);
  return 0;
}

// ---- k-means update -------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void kmeans_accum_kernel(const int8_t* __restrict__ X, int64_t n, int D,
                                                           const int* __restrict__ labels,
                                                           int* __restrict__ sums, int* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nwaves) {
    const int l = labels[i];
    for (int c = lane; c < D; c += 64) atomicAdd(sums + (int64_t)l * D + c, (int)X[i * D + c]);
    if (lane == 0) atomicAdd(counts + l, 1);
  }
}

// f_c = RN(1 / RN(sqrt(x))) for an integer-valued float 0 < x < 2^24, exactly as numpy's IEEE
// float32 computes it.  The device sqrtf / reciprocal are not relied on for the last bit (a 1-ulp
// difference was measured on the k-means path): each step is fixed against the midpoints to its
// float neighbours, with products that are exact in f64 (<= 50 significant bits).
__device__ __forceinline__ float f32_up(float v) { return __uint_as_float(__float_as_uint(v) + 1u); }
__device__ __forceinline__ float f32_dn(float v) { return __uint_as_float(__float_as_uint(v) - 1u); }
__device__ __forceinline__ float cr_inv_sqrt_int(float x) {
  float y = (float)sqrt((double)x);
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // y = RN(sqrt(x)): no midpoint squares to an integer, no ties
    const double mu = 0.5 * ((double)y + (double)f32_up(y)), md = 0.5 * ((double)y + (double)f32_dn(y));
    if ((double)x > mu * mu)
      y = f32_up(y);
    else if ((double)x < md * md)
      y = f32_dn(y);
  }
  float r = (float)(1.0 / (double)y);
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // r = RN(1 / y): compare 1 with midpoint * y (exact in f64)
    const double pu = 0.5 * ((double)r + (double)f32_up(r)) * (double)y;
    const double pd = 0.5 * ((double)r + (double)f32_dn(r)) * (double)y;
    if (pu < 1.0 || (pu == 1.0 && (__float_as_uint(r) & 1u)))
      r = f32_up(r);
    else if (pd > 1.0 || (pd == 1.0 && (__float_as_uint(r) & 1u)))
      r = f32_dn(r);
  }
  return r;
}

// qc_c = clamp(rint(f32(sum) * (127 / f32(amax))), ±127) where the cluster is non-empty and
// amax > 0 (else unchanged); then f_c = 1 / sqrt(f32(sum qc²)).  One wave per centroid.
__global__ __launch_bounds__(256) void centroid_update_kernel(const int* __restrict__ sums,
                                                              const int* __restrict__ counts, int m, int D,
                                                              int8_t* __restrict__ qc, float* __restrict__ fc) {
  const int lane = threadIdx.x & 63;
  const int c = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (c >= m) return;
  if (sums) {
    int amax = 0;
    for (int d = lane; d < D; d += 64) amax = max(amax, abs(sums[(int64_t)c * D + d]));
#pragma unroll
    for (int off = 32; off; off >>= 1) amax = max(amax, __shfl_xor(amax, off));
    if (counts[c] > 0 && amax > 0) {
      const float sc = __fdiv_rn(127.f, (float)amax);
      for (int d = lane; d < D; d += 64) {
        const float q = rintf(__fmul_rn((float)sums[(int64_t)c * D + d], sc));
        qc[(int64_t)c * D + d] = (int8_t)fminf(fmaxf(q, -127.f), 127.f);
      }
    }
  }
  int n2 = 0;
  for (int d = lane; d < D; d += 64) {
    const int v = qc[(int64_t)c * D + d];
    n2 += v * v;
  }
#pragma unroll
  for (int off = 32; off; off >>= 1) n2 += __shfl_xor(n2, off);
  if (lane == 0) fc[c] = n2 > 0 ? cr_inv_sqrt_int((float)n2) : 0.f;
}

// initial centroids: qc_j = codes row j * step
__global__ void init_centroids_kernel(const int8_t* __restrict__ codes, int64_t step, int m, int D,
                                      int8_t* __restrict__ qc) {
  const int64_t total = (int64_t)m * (D >> 4);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i / (D >> 4), c = i - j * (D >> 4);
    *(uint4*)(qc + j * D + c * 16) = *(const uint4*)(codes + j * step * D + c * 16);
  }
}

void launch_init_centroids(const int8_t* codes, int64_t step, int m, int D, int8_t* qc, hipStream_t st) {
  const int64_t total = (int64_t)m * (D >> 4);
  hipLaunchKernelGGL(init_centroids_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0,
                     st, codes, step, m, D, qc);
}

void launch_kmeans_accum(const int8_t* X, int64_t n, int D, const int* labels, int* sums, int* counts,
                         hipStream_t st) {
  const int blocks = (int)std::min<int64_t>((std::max<int64_t>(n, 1) + 3) / 4, 8192);
  hipLaunchKernelGGL(kmeans_accum_kernel, dim3(blocks), dim3(256), 0, st, X, n, D, labels, sums, counts);
}

void launch_centroid_update(const int* sums, const int* counts, int m, int D, int8_t* qc, float* fc, hipStream_t st) {
  hipLaunchKernelGGL(centroid_update_kernel, dim3((m + 3) / 4), dim3(256), 0, st, sums, counts, m, D, qc, fc);
}

// ---- posting lists ---------------------------------------------------------------------------------
__global__ void iota_kernel(int* __restrict__ v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (int)i;
}

__global__ void histogram_kernel(const int* __restrict__ labels, int64_t n, int* __restrict__ counts) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(counts + labels[i], 1);
}

// offsets[0..m] = exclusive scan of counts (one block)
__global__ __launch_bounds__(1024) void offsets_kernel(const int* __restrict__ counts, int m,
                                                       int64_t* __restrict__ off) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (m + 1023) / 1024;
  const int b = t * per, e = min(m, b + per);
  int64_t s = 0;
  for (int i = b; i < e; ++i) s += counts[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int i = b; i < e; ++i) {
    off[i] = run;
    run += counts[i];
  }
  if (t == 1023) off[m] = part[1023];
}

// list-order copy of codes and scales: dst row p = src row ids[p] (one wave per row).  Round 6: the
// list-order codes are stored in 64-row blocks, chunk-major: 16-B chunk c of row p at
// (p / 64) * 64 D + c * 1024 + (p % 64) * 16, so the list scan's lane-per-row loads are 1-KB runs
// (kBlockRows rows of one chunk) and every lane holds a whole row's dot (list_scan_kernel).
__global__ __launch_bounds__(256) void gather_rows_kernel(const int8_t* __restrict__ codes,
                                                          const float* __restrict__ inv,
                                                          const int* __restrict__ ids, int64_t n, int D,
                                                          int8_t* __restrict__ dcodes, float* __restrict__ dinv) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int nch = D >> 4;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < n; p += nwaves) {
    const int64_t src = ids[p];
    for (int c = lane; c < nch; c += 64)
      *(uint4*)(dcodes + (p >> 6) * 64 * D + c * 1024 + (p & 63) * 16) = *(const uint4*)(codes + src * D + c * 16);
    if (lane == 0) dinv[p] = inv[src];
  }
}

size_t sort_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                            (const int*)nullptr, (int*)nullptr, (size_t)n, 0u, 32u);
  return bytes;
}

// ids sorted by (label, row): stable LSD radix sort of (label, row id) pairs
int launch_build_lists(const int* labels, int64_t n, int m, const int8_t* codes, const float* inv, int D,
                       unsigned* keys_tmp, int* vals_tmp, unsigned* keys_out, int* ids_out, void* sort_tmp,
                       size_t sort_tmp_bytes, int* counts, int64_t* off, int8_t* dcodes, float* dinv,
                       hipStream_t st) {
  if (hipMemsetAsync(counts, 0, (size_t)m * sizeof(int), st) != hipSuccess) return -2;
  if (n > 0) {
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(histogram_kernel, dim3(blocks), dim3(256), 0, st, labels, n, counts);
    hipLaunchKernelGGL(iota_kernel, dim3(blocks), dim3(256), 0, st, vals_tmp, n);
    if (hipMemcpyAsync(keys_tmp, labels, (size_t)n * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return -2;
    unsigned end_bit = 1;
    while ((1u << end_bit) < (unsigned)m) ++end_bit;
    size_t tb = sort_tmp_bytes;
    if (rocprim::radix_sort_pairs(sort_tmp, tb, (const unsigned*)keys_tmp, keys_out, (const int*)vals_tmp, ids_out,
                                  (size_t)n, 0u, end_bit, st) != hipSuccess)
      return -3;
  }
  hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(1024), 0, st, counts, m, off);
  if (n > 0) {
    const int blocks = (int)std::min<int64_t>((n + 3) / 4, 8192);
    hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(256), 0, st, codes, inv, ids_out, n, D, dcodes, dinv);
  }
  return 0;
}

// ---- search: (query, probe) pairs grouped by list ---------------------------------------------------
// pair p = q * nprobe + j probes list probes[p]; out: pair_off[0..m] (CSR by list), pairs[].
constexpr int kMaxListsGroup = 16384;
__global__ __launch_bounds__(1024) void group_pairs_kernel(const int64_t* __restrict__ probes, int P, int m,
                                                           int* __restrict__ pair_off, int* __restrict__ pairs) {
  __shared__ int cnt[kMaxListsGroup];
  __shared__ int part[1024];
  const int t = threadIdx.x;
  for (int i = t; i < m; i += 1024) cnt[i] = 0;
  __syncthreads();
  for (int p = t; p < P; p += 1024) atomicAdd(&cnt[(int)probes[p]], 1);
  __syncthreads();
  const int per = (m + 1023) / 1024;
  const int b = t * per, e = min(m, b + per);
  int s = 0;
  for (int i = b; i < e; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - s;
  for (int i = b; i < e; ++i) {
    const int c = cnt[i];
    pair_off[i] = run;
    cnt[i] = run;  // becomes the list's cursor
    run += c;
  }
  if (t == 1023) pair_off[m] = part[1023];
  __syncthreads();
  for (int p = t; p < P; p += 1024) pairs[atomicAdd(&cnt[(int)probes[p]], 1)] = p;
}

// Posting-list scan.  Grid (list, split): block (L, s) takes the 64-row groups s*4 + w,
// s*4 + w + 4*S, ... of list L (S splits balance long lists over the chip); the queries probing
// it (pairs) in batches of QB staged in LDS; every wave streams rows (16 lanes per row, 16-byte
// chunks j, j+16, ..), v_dot4_i32_i8 against each staged query, DPP row sum, and keeps one
// top-K list per query.  Candidates: cand[((q * nprobe + j) * S + s) * 4 + wave][K] (every pair
// of every list is written, empty lists too).
constexpr int kQB = 8;
constexpr int kSeedChunks = 2;

// The K best of a wave's kept candidates per query, exactly as the sorted list would hold them: (score desc,
// id asc), each query's K in lanes 0..K-1, sorted, and the list's threshold set (WaveList).  v = the K-th
// largest orderable score (bitwise search on ballot counts); ties at v are taken by the smallest ids (a second
// bitwise search over the tied ids), so the set is the list's set whatever the order the rows came in.
// Wave-local (LDS rows of this wave only).
template <int K, int QB, int NCH>
__device__ __forceinline__ void seed_lists(float (&ka)[QB][NCH], int (&kg)[NCH], WaveList<K> (&lst)[QB], int w) {
  __shared__ float ssa[4][K];
  __shared__ int ssr[4][K];
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int qi = 0; qi < QB; ++qi) {
    uint32_t key[NCH];
    int nvalid = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      key[c] = ka[qi][c] == ka[qi][c] ? ord_f32(ka[qi][c]) : 0u;
      nvalid += (int)__popcll(__ballot(key[c] != 0u));
    }
    uint32_t v = 0u;
    if (nvalid > K)
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c1 = v | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int c = 0; c < NCH; ++c) cnt += (int)__popcll(__ballot(key[c] >= c1));
        v = cnt >= K ? c1 : v;
      }
    int room = K;
#pragma unroll
    for (int c = 0; c < NCH; ++c) room -= (int)__popcll(__ballot(key[c] > v));
    // ties at v (v > 0 only): the room smallest ids, gid <= g2
    uint32_t g2 = 0u;
    if (v != 0u) {
      int ntie = 0;
#pragma unroll
      for (int c = 0; c < NCH; ++c) ntie += (int)__popcll(__ballot(key[c] == v));
      if (ntie > room) {
        // g2 = the room-th smallest tied id: the largest value with fewer than room tied ids below it
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t c1 = g2 | (1u << bit);
          int cnt = 0;
#pragma unroll
          for (int c = 0; c < NCH; ++c) cnt += (int)__popcll(__ballot(key[c] == v && (uint32_t)kg[c] < c1));
          g2 = cnt < room ? c1 : g2;
        }
      } else {
        g2 = 0xffffffffu;
      }
    }
    int base = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const bool keep = key[c] > v || (v != 0u && key[c] == v && (uint32_t)kg[c] <= g2);
      const uint64_t kb = __ballot(keep);
      const int p =
          base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(kb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)kb, 0u));
      if (keep) {
        ssa[w][p] = ka[qi][c];
        ssr[w][p] = kg[c];
      }
      base += (int)__popcll(kb);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float ls = lane < base ? ssa[w][lane] : -__builtin_inff();
    int lr = lane < base ? ssr[w][lane] : kEmptyRow;
    __builtin_amdgcn_wave_barrier();  // (read before the next query's compaction rewrites the rows)
#pragma unroll
    for (int kk = 2; kk <= K; kk <<= 1)
#pragma unroll
      for (int jj = kk >> 1; jj > 0; jj >>= 1) {
        const float ps = __shfl_xor(ls, jj);
        const int pr = __shfl_xor(lr, jj);
        const bool lower = (lane & jj) == 0, desc = (lane & kk) == 0;
        const bool mine = better(ls, lr, ps, pr);
        if (lower == desc ? !mine : mine) {
          ls = ps;
          lr = pr;
        }
      }
    lst[qi].ls = lane < K ? ls : -__builtin_inff();
    lst[qi].lr = lane < K ? lr : kEmptyRow;
    lst[qi].ts = readlane_f(ls, K - 1);
    lst[qi].tr = readlane_i(lr, K - 1);
  }
}

template <int K, int NC>
__global__ __launch_bounds__(256) void list_scan_kernel(const int8_t* __restrict__ codes, const float* __restrict__ inv,
                                                        const int* __restrict__ ids, const int64_t* __restrict__ off,
                                                        const int* __restrict__ pair_off, const int* __restrict__ pairs,
                                                        int nprobe, const int8_t* __restrict__ qq,
                                                        const float* __restrict__ qinv, float* __restrict__ cand_s,
                                                        int* __restrict__ cand_r) {
  constexpr int D = NC * 256, NCH = D / 16;  // 16-B chunks per row
  // Round 6: one lane per row.  The codes are in 64-row blocks, chunk-major (gather_rows_kernel), so a wave's
  // load of chunk c of its 64 rows is one 1-KB run; the batch's queries are wave-uniform and come through
  // scalar loads (SGPR operands of v_dot4), so no LDS reads, and every lane ends with its row's whole dot
  // for each query (no cross-lane sums).  Before, 16 lanes shared a row: per 4 rows a wave read 8 KB of
  // staged queries from LDS and summed 8 dots over 16 lanes (DPP), the list scan at 5.3 TB/s.
  constexpr int G = 4;  // chunks per load group (double-buffered)
  static_assert(NCH % G == 0, "chunk groups");
  constexpr int NG = NCH / G;
  __shared__ float qf[kQB];
  const int L = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
  const int p0 = pair_off[L], p1 = pair_off[L + 1];
  if (p0 == p1) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t r0 = off[L], r1 = off[L + 1];
  for (int pb = p0; pb < p1; pb += kQB) {
    const int nb = min(kQB, p1 - pb);
    const uint4* qv[kQB];
#pragma unroll
    for (int qi = 0; qi < kQB; ++qi)
      qv[qi] = (const uint4*)(qq + (int64_t)(pairs[pb + (qi < nb ? qi : 0)] / nprobe) * D);
    if (tid < kQB) qf[tid] = tid < nb ? qinv[pairs[pb + tid] / nprobe] : 0.f;
    __syncthreads();
    WaveList<K> lst[kQB];
#pragma unroll
    for (int qi = 0; qi < kQB; ++qi) lst[qi].init();
    // Round 6: a wave's first kSeedChunks 64-row chunks are kept in registers (score per lane, chunk and
    // query; the id per lane and chunk) and seed each query's sorted list by one selection (seed_lists), the
    // later chunks go through the list inserts.  A config-5 wave streams ~3 chunks of a list per batch, so the
    // inserts of its first chunks — nearly every candidate, the list still empty — were most of them.
    float ka[kQB][kSeedChunks];
    int kg[kSeedChunks];
    int nch = 0;  // chunks this wave has scored in this batch (wave-uniform)
#pragma unroll
    for (int c = 0; c < kSeedChunks; ++c) {
#pragma unroll
      for (int qi = 0; qi < kQB; ++qi) ka[qi][c] = __builtin_nanf("");
      kg[c] = kEmptyRow;
    }
    for (int64_t base = r0 + (int64_t)(sp * 4 + w) * 64; base < r1; base += 256 * S) {
      const int64_t crow = base + lane;
      const bool valid = crow < r1;
      const int64_t cr = valid ? crow : r0;  // in-list row (never past the list)
      const int8_t* rp = codes + (cr >> 6) * (64 * D) + (cr & 63) * 16;  // chunk c at rp + c * 1024
      int acc[kQB];
#pragma unroll
      for (int qi = 0; qi < kQB; ++qi) acc[qi] = 0;
      uint4 va[G], vb[G];
#pragma unroll
      for (int c = 0; c < G; ++c) va[c] = *(const uint4*)(rp + c * 1024);
#pragma unroll
      for (int cg = 0; cg < NG; ++cg) {
        uint4(&cur)[G] = (cg & 1) ? vb : va;
        uint4(&nxt)[G] = (cg & 1) ? va : vb;
        if (cg + 1 < NG) {
#pragma unroll
          for (int c = 0; c < G; ++c) nxt[c] = *(const uint4*)(rp + ((cg + 1) * G + c) * 1024);
        }
#pragma unroll
        for (int qi = 0; qi < kQB; ++qi) {
          if (qi < nb) {
#pragma unroll
            for (int c = 0; c < G; ++c) {
              const uint4 q = qv[qi][cg * G + c];
              acc[qi] = __builtin_amdgcn_sdot4((int)cur[c].x, (int)q.x, acc[qi], false);
              acc[qi] = __builtin_amdgcn_sdot4((int)cur[c].y, (int)q.y, acc[qi], false);
              acc[qi] = __builtin_amdgcn_sdot4((int)cur[c].z, (int)q.z, acc[qi], false);
              acc[qi] = __builtin_amdgcn_sdot4((int)cur[c].w, (int)q.w, acc[qi], false);
            }
          }
        }
      }
      float cand[kQB];  // |dot| <= 768 * 127 * 127 < 2^24: exact in f32, the value the 16-lane sum had
#pragma unroll
      for (int qi = 0; qi < kQB; ++qi) cand[qi] = (float)acc[qi];
      const float ir = inv[cr];
      const int gid = ids[cr];
      if (nch < kSeedChunks) {
#pragma unroll
        for (int c = 0; c < kSeedChunks; ++c)
          if (c == nch) {
#pragma unroll
            for (int qi = 0; qi < kQB; ++qi)
              ka[qi][c] = valid && qi < nb ? __fmul_rn(cand[qi], __fmul_rn(ir, qf[qi])) : __builtin_nanf("");
            kg[c] = gid;
          }
        if (++nch == kSeedChunks) seed_lists<K, kQB, kSeedChunks>(ka, kg, lst, w);
      } else {
#pragma unroll
        for (int qi = 0; qi < kQB; ++qi)
          if (qi < nb) lst[qi].offer(__fmul_rn(cand[qi], __fmul_rn(ir, qf[qi])), gid, valid);
      }
    }
    if (nch < kSeedChunks) seed_lists<K, kQB, kSeedChunks>(ka, kg, lst, w);  // (fewer chunks than kept)
    if (lane < K) {
#pragma unroll
      for (int qi = 0; qi < kQB; ++qi) {
        if (qi < nb) {
          const int64_t o = (((int64_t)pairs[pb + qi] * S + sp) * 4 + w) * K + lane;
          cand_s[o] = lst[qi].ls;
          cand_r[o] = lst[qi].lr;
        }
      }
    }
    __syncthreads();  // qs reused by the next batch
  }
}

int list_k(int k) { return k <= 4 ? 4 : (k <= 16 ? 16 : (k <= 64 ? 64 : -1)); }

int launch_list_scan(int K, int D, int m, int splits, const int8_t* codes, const float* inv, const int* ids, const int64_t* off,
                     const int* pair_off, const int* pairs, int nprobe, const int8_t* qq, const float* qinv,
                     float* cs, int* cr, hipStream_t st) {
#define RFX_LS(KV, NCV)                                                                                     \
  if (K == KV && D == NCV * 256) {                                                                          \
    hipLaunchKernelGGL((list_scan_kernel<KV, NCV>), dim3(m, splits), dim3(256), 0, st, codes, inv, ids, off,  \
                       pair_off, pairs, nprobe, qq, qinv, cs, cr);                                          \
    return 0;                                                                                               \
  }
  RFX_LS(4, 1) RFX_LS(4, 2) RFX_LS(4, 3) RFX_LS(4, 4)
  RFX_LS(16, 1) RFX_LS(16, 2) RFX_LS(16, 3) RFX_LS(16, 4)
  RFX_LS(64, 1) RFX_LS(64, 2) RFX_LS(64, 3) RFX_LS(64, 4)
#undef RFX_LS
  return -1;
}

// ---- probe selection: each query's nprobe best coarse scores (round 6) ----------------------------
// One 256-thread block per query, up to kProbeMaxLists scores held in registers (16 per thread, list
// c = tid + 256 i).  v = the nprobe-th largest orderable score by a bitwise search on block-wide ballot
// counts; ties at v are taken by the smallest list ids (a second bitwise search over the tied ids): the
// set the merge kernel's (score desc, id asc) top-nprobe returns.  The probes are written in no particular
// order (the pairs are grouped by list next, and every later step is order-free).
constexpr int kProbeMaxLists = 4096;
__global__ __launch_bounds__(256) void probe_select_kernel(const float* __restrict__ S, int m, int nprobe,
                                                           float* __restrict__ ps, int64_t* __restrict__ pid) {
  constexpr int PT = kProbeMaxLists / 256;
  __shared__ int wc[2][4];
  __shared__ int npos;
  const int tid = threadIdx.x, w = tid >> 6;
  const int64_t q = blockIdx.x;
  uint32_t key[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int c = tid + 256 * i;
    key[i] = c < m ? ord_f32(S[q * m + c]) : 0u;
  }
  if (tid == 0) npos = 0;
  // block-wide count of the keys meeting pred (two LDS slots alternate, so one barrier per count)
  int par = 0;
  auto block_count = [&](auto pred) {
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i) cnt += (int)__popcll(__ballot(pred(i)));
    if ((tid & 63) == 0) wc[par][w] = cnt;
    __syncthreads();
    const int t = wc[par][0] + wc[par][1] + wc[par][2] + wc[par][3];
    par ^= 1;
    return t;
  };
  uint32_t v = 0u;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t c1 = v | (1u << bit);
    if (block_count([&](int i) { return key[i] >= c1; }) >= nprobe) v = c1;
  }
  const int room = nprobe - block_count([&](int i) { return key[i] > v; });
  const int ntie = block_count([&](int i) { return key[i] == v; });
  uint32_t g2 = 0xffffffffu;  // tied ids <= g2 are kept
  if (ntie > room) {
    g2 = 0u;
    for (int bit = 12; bit >= 0; --bit) {  // ids < 4096
      const uint32_t c1 = g2 | (1u << bit);
      if (block_count([&](int i) { return key[i] == v && (uint32_t)(tid + 256 * i) < c1; }) < room) g2 = c1;
    }
  }
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int c = tid + 256 * i;
    const bool keep = c < m && (key[i] > v || (key[i] == v && (uint32_t)c <= g2));
    if (keep) {
      const int o = atomicAdd(&npos, 1);
      ps[q * nprobe + o] = S[q * m + c];
      pid[q * nprobe + o] = c;
    }
  }
}

int launch_probe_select(const float* S, int64_t nq, int m, int nprobe, float* ps, int64_t* pid, hipStream_t st) {
  if (m > kProbeMaxLists || nprobe < 1 || nprobe > m || nq <= 0) return -1;
  hipLaunchKernelGGL(probe_select_kernel, dim3((unsigned)nq), dim3(256), 0, st, S, m, nprobe, ps, pid);
  return 0;
}

int launch_group_pairs(const int64_t* probes, int P, int m, int* pair_off, int* pairs, hipStream_t st) {
  if (m > kMaxListsGroup) return -1;
  hipLaunchKernelGGL(group_pairs_kernel, dim3(1), dim3(1024), 0, st, probes, P, m, pair_off, pairs);
  return 0;
}

}  // namespace ivf
}  // namespace rfx

namespace rfx {
namespace ivf {

// ---- exact re-rank of IVF candidates against the original rows -----------------------------------
// One block per query, one wave per candidate (strided): f32 dot of the query and the candidate's
// original row (bf16 / f16 / f32, e.g. the brute-force store's buffer), wave reduction.  Rows < 0
// (padding) stay -1 with score -inf, which the merge skips.  Row-sharded use (rfx_rerank_candidates):
// the candidates are global rows, X holds rows [row_lo, row_lo + n_rows); the others are padding here.
template <int DTQ, int DTX>
__global__ __launch_bounds__(256) void rerank_kernel(const void* __restrict__ Q, const void* __restrict__ X, int D,
                                                     const int64_t* __restrict__ cand, int kc, int64_t row_lo,
                                                     int64_t n_rows, float* __restrict__ out_s,
                                                     int64_t* __restrict__ out_r) {
  const int64_t q = blockIdx.x;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = w; c < kc; c += 4) {
    const int64_t r = cand[q * kc + c];
    const int64_t lr = r - row_lo;
    const bool own = r >= 0 && lr >= 0 && lr < n_rows;
    float acc = 0.f;
    if (own)
      for (int d = lane; d < D; d += 64) acc = fmaf(load_elem<DTQ>(Q, q * D + d), load_elem<DTX>(X, lr * D + d), acc);
#pragma unroll
    for (int off = 32; off; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
      out_s[q * kc + c] = own ? acc : -__builtin_inff();
      out_r[q * kc + c] = own ? r : -1;  // (negative rows are never live in the merge)
    }
  }
}

int launch_rerank(const void* Q, int dtq, const void* X, int dtx, int D, const int64_t* cand, int64_t nq, int kc,
                  float* out_s, int64_t* out_r, hipStream_t st, int64_t row_lo, int64_t n_rows) {
  if (nq <= 0) return 0;
#define RFX_RR(A, B)                                                                                        \
  if (dtq == A && dtx == B) {                                                                               \
    hipLaunchKernelGGL((rerank_kernel<A, B>), dim3((unsigned)nq), dim3(256), 0, st, Q, X, D, cand, kc, row_lo, \
                       n_rows, out_s, out_r);                                                               \
    return 0;                                                                                               \
  }
  RFX_RR(RFX_F32, RFX_F32) RFX_RR(RFX_F32, RFX_BF16) RFX_RR(RFX_F32, RFX_F16)
  RFX_RR(RFX_BF16, RFX_F32) RFX_RR(RFX_BF16, RFX_BF16) RFX_RR(RFX_BF16, RFX_F16)
  RFX_RR(RFX_F16, RFX_F32) RFX_RR(RFX_F16, RFX_BF16) RFX_RR(RFX_F16, RFX_F16)
#undef RFX_RR
  return -1;
}

}  // namespace ivf
}  // namespace rfx
