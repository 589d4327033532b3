// vmm_probe.hip — round 6 probe of HIP virtual memory on the MI355X box (zero-copy union views):
// the allocation granularities, whether two physical allocations mapped back to back in one reserved range
// alias their own mappings (a write through one mapping is read through the other), and the streaming read
// rate through a VMM mapping against a hipMalloc buffer of the same size.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/r06/vmm_probe tools/r06/vmm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                        \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (uint32_t)i;
}
// streaming read: 16 B per lane per step, xor-folded into one word per block (so nothing is optimised away)
__global__ void stream_read(const uint4* p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  CK(hipSetDevice(0));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity minimum %zu recommended %zu\n", gmin, grec);
  const size_t g = grec;
  const size_t part = ((size_t)4 << 30) / g * g;  // two 4-GiB physical allocations
  hipMemGenericAllocationHandle_t h[2];
  void* own[2];
  void* cat = nullptr;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (int i = 0; i < 2; ++i) {
    CK(hipMemCreate(&h[i], part, &prop, 0));
    CK(hipMemAddressReserve(&own[i], part, g, nullptr, 0));
    CK(hipMemMap(own[i], part, 0, h[i], 0));
    CK(hipMemSetAccess(own[i], part, &acc, 1));
  }
  CK(hipMemAddressReserve(&cat, 2 * part, g, nullptr, 0));
  for (int i = 0; i < 2; ++i) CK(hipMemMap((uint8_t*)cat + i * part, part, 0, h[i], 0));
  CK(hipMemSetAccess(cat, 2 * part, &acc, 1));
  // aliasing: write through the own mappings, read through the concatenated one
  fill<<<1024, 256>>>((uint32_t*)own[0], part / 4, 7u);
  fill<<<1024, 256>>>((uint32_t*)own[1], part / 4, 1000000007u);
  CK(hipDeviceSynchronize());
  uint32_t a[2], b[2];
  CK(hipMemcpy(a, (uint8_t*)cat + 4 * 12345, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b, (uint8_t*)cat + part + 4 * 777, 4, hipMemcpyDeviceToHost));
  printf("alias %s (%u %u, want %u %u)\n", (a[0] == 7u + 12345u && b[0] == 1000000007u + 777u) ? "ok" : "BROKEN", a[0], b[0],
         7u + 12345u, 1000000007u + 777u);
  // streaming read rate: hipMalloc buffer vs the concatenated VMM range (8 GiB each)
  void* plain = nullptr;
  CK(hipMalloc(&plain, 2 * part));
  fill<<<1024, 256>>>((uint32_t*)plain, 2 * part / 4, 3u);
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, 1 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      const uint4* p = (const uint4*)(which ? cat : plain);
      stream_read<<<256 * 8, 512>>>(p, 2 * part / 16, out);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) stream_read<<<256 * 8, 512>>>(p, 2 * part / 16, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("stream %s: %.1f GB/s\n", which ? "vmm-concat" : "hipMalloc ", 5.0 * 2 * part / (ms * 1e-3) / 1e9);
    }
  }
  for (int i = 0; i < 2; ++i) {
    CK(hipMemUnmap((uint8_t*)cat + i * part, part));
    CK(hipMemUnmap(own[i], part));
    CK(hipMemAddressFree(own[i], part));
  }
  CK(hipMemAddressFree(cat, 2 * part));
  // the physical memory lives until every mapping is gone and the handle is released
  for (int i = 0; i < 2; ++i) CK(hipMemRelease(h[i]));
  CK(hipFree(plain));
  printf("done\n");
  return 0;
}
