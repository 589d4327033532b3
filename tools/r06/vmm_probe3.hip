// vmm_probe3.hip — round 6: does a virtual-memory range that is unmapped, released and then reserved again
// (the same address, new physical memory) read the NEW memory in kernels?  (librfx's index tests failed with
// virtual-memory rows after many create / destroy cycles; vmm_probe2's single-allocation checks all pass.)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (uint32_t)i;
}
__global__ void copyk(const uint32_t* s, uint32_t* d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

int main(int argc, char** argv) {
  const bool keep_va = argc > 1;  // never free the address ranges (a fresh address every time)
  (void)hipSetDevice(0);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  const size_t n = (size_t)4 << 20, bytes = n * 4;
  uint32_t* plain = nullptr;
  (void)hipMalloc(&plain, bytes);
  std::vector<uint32_t> host(n), got(n);
  int bad_rounds = 0, reused = 0;
  void* prev = nullptr;
  for (int round = 0; round < 40; ++round) {
    hipMemGenericAllocationHandle_t h;
    void* va = nullptr;
    if (hipMemCreate(&h, bytes, &prop, 0) != hipSuccess || hipMemAddressReserve(&va, bytes, 4096, nullptr, 0) != hipSuccess ||
        hipMemMap(va, bytes, 0, h, 0) != hipSuccess || hipMemSetAccess(va, bytes, &acc, 1) != hipSuccess) {
      printf("alloc failed in round %d\n", round);
      return 1;
    }
    reused += va == prev;
    prev = va;
    const uint32_t v = 1000u * (uint32_t)round;
    if (round & 1) {
      for (size_t i = 0; i < n; ++i) host[i] = v + (uint32_t)i;
      (void)hipMemcpy(va, host.data(), bytes, hipMemcpyHostToDevice);  // SDMA write
    } else {
      fill<<<512, 256>>>((uint32_t*)va, n, v);  // kernel write
    }
    copyk<<<512, 256>>>((const uint32_t*)va, plain, n);
    (void)hipMemcpy(got.data(), plain, bytes, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += got[i] != v + (uint32_t)i;
    if (bad) {
      ++bad_rounds;
      printf("round %d (%s write): %zu of %zu words stale/wrong, va %p\n", round, (round & 1) ? "H2D" : "kernel", bad, n, va);
    }
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap(va, bytes);
    if (!keep_va) (void)hipMemAddressFree(va, bytes);
    (void)hipMemRelease(h);
  }
  printf("%s: %d bad rounds of 40, address reused %d times\n", keep_va ? "fresh addresses" : "freed addresses", bad_rounds,
         reused);
  return 0;
}
