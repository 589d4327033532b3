// vmm_probe2.hip — round 6: which HIP operations on virtual-memory mappings give wrong data on the box
// (the index tests failed with librfx's rows in hipMemCreate + hipMemMap memory, and passed with RFX_VMM=0).
// Each check writes a pattern through one path and reads it back through another.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (uint32_t)i;
}
__global__ void copyk(const uint32_t* s, uint32_t* d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

static void* vmm(size_t bytes, hipMemGenericAllocationHandle_t* h) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  void* va = nullptr;
  if (hipMemCreate(h, bytes, &prop, 0) != hipSuccess) return nullptr;
  if (hipMemAddressReserve(&va, bytes, 4096, nullptr, 0) != hipSuccess) return nullptr;
  if (hipMemMap(va, bytes, 0, *h, 0) != hipSuccess) return nullptr;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(va, bytes, &acc, 1) != hipSuccess) return nullptr;
  return va;
}

static int check(const char* what, const std::vector<uint32_t>& got, const std::vector<uint32_t>& want) {
  size_t bad = 0, first = (size_t)-1;
  for (size_t i = 0; i < got.size(); ++i)
    if (got[i] != want[i]) {
      if (first == (size_t)-1) first = i;
      ++bad;
    }
  if (bad)
    printf("%-44s BAD: %zu of %zu words differ (first at %zu: %08x want %08x)\n", what, bad, got.size(), first, got[first],
           want[first]);
  else
    printf("%-44s ok\n", what);
  return bad ? 1 : 0;
}

int main() {
  CK(hipSetDevice(0));
  const size_t n = (size_t)16 << 20, bytes = n * 4;  // 64 MiB
  hipMemGenericAllocationHandle_t ha, hb;
  uint32_t* a = (uint32_t*)vmm(bytes, &ha);
  uint32_t* b = (uint32_t*)vmm(bytes, &hb);
  if (!a || !b) {
    printf("vmm alloc failed\n");
    return 1;
  }
  uint32_t* plain = nullptr;
  CK(hipMalloc(&plain, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint32_t> host(n), got(n), want(n);
  int bad = 0;
  // 1. kernel write, D2H read
  fill<<<1024, 256, 0, st>>>(a, n, 5u);
  CK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; ++i) want[i] = 5u + (uint32_t)i;
  CK(hipMemcpy(got.data(), a, bytes, hipMemcpyDeviceToHost));
  bad += check("kernel write -> hipMemcpy D2H", got, want);
  // 2. hipMemsetD32Async, D2H read
  CK(hipMemsetD32Async((hipDeviceptr_t)a, 0x7fc00000, n, st));
  CK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; ++i) want[i] = 0x7fc00000u;
  CK(hipMemcpy(got.data(), a, bytes, hipMemcpyDeviceToHost));
  bad += check("hipMemsetD32Async -> D2H", got, want);
  // 3. hipMemsetAsync (bytes), kernel read into plain, D2H
  CK(hipMemsetAsync(a, 0, bytes, st));
  copyk<<<1024, 256, 0, st>>>(a, plain, n);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(got.data(), plain, bytes, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; ++i) want[i] = 0u;
  bad += check("hipMemsetAsync -> kernel read", got, want);
  // 4. H2D async, kernel read
  for (size_t i = 0; i < n; ++i) host[i] = 0x1234u ^ (uint32_t)(i * 2654435761u);
  CK(hipMemcpyAsync(a, host.data(), bytes, hipMemcpyHostToDevice, st));
  copyk<<<1024, 256, 0, st>>>(a, plain, n);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(got.data(), plain, bytes, hipMemcpyDeviceToHost));
  bad += check("hipMemcpyAsync H2D -> kernel read", got, host);
  // 5. D2D async vmm -> vmm (the growth copy), kernel read
  CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, st));
  copyk<<<1024, 256, 0, st>>>(b, plain, n);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(got.data(), plain, bytes, hipMemcpyDeviceToHost));
  bad += check("hipMemcpyAsync D2D vmm->vmm -> kernel read", got, host);
  // 6. D2D plain -> vmm, D2H
  fill<<<1024, 256, 0, st>>>(plain, n, 77u);
  CK(hipMemcpyAsync(b, plain, bytes, hipMemcpyDeviceToDevice, st));
  CK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; ++i) want[i] = 77u + (uint32_t)i;
  CK(hipMemcpy(got.data(), b, bytes, hipMemcpyDeviceToHost));
  bad += check("hipMemcpyAsync D2D plain->vmm -> D2H", got, want);
  // 7. null-stream (legacy) memcpy H2D then kernel on another stream after a device sync
  CK(hipMemcpy(a, host.data(), bytes, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  copyk<<<1024, 256, 0, st>>>(a, plain, n);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(got.data(), plain, bytes, hipMemcpyDeviceToHost));
  bad += check("hipMemcpy H2D (sync) -> kernel read", got, host);
  // 8. small offset copies (rows appended one by one) H2D at unaligned row offsets
  for (size_t r = 0; r < 64; ++r)
    CK(hipMemcpyAsync((uint8_t*)a + r * 1536 + 4096 * 3, host.data() + r * 384, 1536, hipMemcpyHostToDevice, st));
  CK(hipStreamSynchronize(st));
  std::vector<uint32_t> g2(64 * 384), w2(host.begin(), host.begin() + 64 * 384);
  CK(hipMemcpy(g2.data(), (uint8_t*)a + 4096 * 3, 64 * 1536, hipMemcpyDeviceToHost));
  bad += check("64 row copies H2D at offsets -> D2H", g2, w2);
  // 9. hipMemcpyAsync D2H async from vmm
  fill<<<1024, 256, 0, st>>>(a, n, 9u);
  CK(hipMemcpyAsync(got.data(), a, bytes, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; ++i) want[i] = 9u + (uint32_t)i;
  bad += check("kernel write -> hipMemcpyAsync D2H", got, want);
  // 10. pointer attributes of a mapped address (what the runtime knows about it)
  hipPointerAttribute_t attr;
  const hipError_t pe = hipPointerGetAttributes(&attr, (uint8_t*)a + 12345);
  printf("hipPointerGetAttributes: %s type %d device %d\n", hipGetErrorString(pe), (int)attr.type, attr.device);
  printf("%s\n", bad ? "SOME CHECKS FAILED" : "all ok");
  return 0;
}
