// rfx_api.hip — C-ABI of librfx (declared in include/rfx.h).
//
// Owns the vector-store storage (one device buffer per index handle) and dispatches the
// kernels.  Everything else (queries, outputs, workspaces) is caller-owned device memory —
// in practice torch tensors allocated by the Python host (rag-foundation_amd/rfx).
//
// Thread-safety: handles live in a process-wide registry; each index has a reader/writer
// lock (search = shared, add/tombstone/reserve = exclusive), matching the concurrency the
// reference's callers generate (<=50 chat threads per process, chat.py:496-521; <=10 ingestion
// jobs per worker, worker.py:125).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cstdlib>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "rfx_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define RFX_HIP(call)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess) return fail(RFX_EDEVICE, "%s: %s", #call, hipGetErrorString(e_));    \
  } while (0)

int esize(int dtype) { return dtype == RFX_F32 ? 4 : 2; }
bool valid_dtype(int dtype) { return dtype == RFX_F32 || dtype == RFX_BF16 || dtype == RFX_F16; }

// ---- index memory: physical allocations mapped through HIP virtual memory ---------------------------------
// An index's rows and its int8 copy each live in ONE physical allocation (hipMemCreate) mapped at a reserved
// address range of their own.  A union view (rfx_union_create; a question over several stores,
// gemini_rag.py:463-469) maps the members' physical allocations back to back into one more range: one
// contiguous [rows][dim] image of all members that IS their memory (no copy; appends and tombstones show
// through).  Sizes are multiples of the recommended granularity (capacity_align below).  Unmapping memory a
// kernel still reads would fault the GPU: every release below follows a device synchronisation.
struct Phys {
  hipMemGenericAllocationHandle_t h{};
  size_t bytes = 0;
  ~Phys() {
    if (bytes) (void)hipMemRelease(h);
  }
};
// An address range is never freed, only unmapped: measured on the box (tools/r06/vmm_probe3.hip), a range that
// is freed and reserved again (the runtime hands back the same address) and mapped to NEW physical memory is
// written wrongly by hipMemcpy host-to-device copies — 19 of 40 rounds had 1.5M of 4M words stale — while fresh
// addresses were right in 40 of 40.  Unmapped ranges cost address space only (a store's growth is geometric).
struct Mapping {
  void* va = nullptr;
  size_t bytes = 0;
  std::vector<std::shared_ptr<Phys>> parts;  // mapped back to back from va
  ~Mapping() {
    size_t off = 0;
    for (auto& p : parts) {
      (void)hipMemUnmap((uint8_t*)va + off, p->bytes);
      off += p->bytes;
    }
  }
};

hipMemAllocationProp vmm_prop(int device) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  return prop;
}

// the recommended granularity of the device, 0 when its virtual memory API is unavailable (or RFX_VMM=0:
// plain hipMalloc, no zero-copy union views)
size_t vmm_granularity(int device) {
  static std::mutex mu;
  static std::map<int, size_t> g;
  std::lock_guard<std::mutex> lk(mu);
  auto it = g.find(device);
  if (it != g.end()) return it->second;
  size_t v = 0;
  const char* e = getenv("RFX_VMM");
  int vmm = 0;
  if (!(e && e[0] == '0') && hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device) == hipSuccess &&
      vmm) {
    const hipMemAllocationProp prop = vmm_prop(device);
    if (hipMemGetAllocationGranularity(&v, &prop, hipMemAllocationGranularityRecommended) != hipSuccess) v = 0;
  }
  g[device] = v;
  return v;
}

// map `parts` back to back into a fresh range (read / write for the device)
int vmm_map(int device, const std::vector<std::shared_ptr<Phys>>& parts, std::shared_ptr<Mapping>& out) {
  auto m = std::make_shared<Mapping>();
  for (auto& p : parts) m->bytes += p->bytes;
  const size_t g = vmm_granularity(device);
  if (!g || m->bytes == 0) return fail(RFX_EUNSUPPORTED, "virtual memory unavailable on device %d", device);
  if (hipMemAddressReserve(&m->va, m->bytes, g, nullptr, 0) != hipSuccess) {
    m->va = nullptr;
    return fail(RFX_ENOMEM, "hipMemAddressReserve(%zu) failed", m->bytes);
  }
  // (never freed: see Mapping)
  size_t off = 0;
  for (auto& p : parts) {
    if (hipMemMap((uint8_t*)m->va + off, p->bytes, 0, p->h, 0) != hipSuccess)
      return fail(RFX_ENOMEM, "hipMemMap(%zu) failed", p->bytes);  // (~Mapping unmaps what was mapped)
    m->parts.push_back(p);
    off += p->bytes;
  }
  hipMemAccessDesc acc = {};
  acc.location = vmm_prop(device).location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(m->va, m->bytes, &acc, 1) != hipSuccess) return fail(RFX_ENOMEM, "hipMemSetAccess failed");
  out = m;
  return RFX_OK;
}

// one physical allocation of `bytes` (a multiple of the granularity) at a range of its own
int vmm_alloc(int device, size_t bytes, std::shared_ptr<Mapping>& out) {
  auto p = std::make_shared<Phys>();
  p->bytes = bytes;
  const hipMemAllocationProp prop = vmm_prop(device);
  if (hipMemCreate(&p->h, bytes, &prop, 0) != hipSuccess) {
    p->bytes = 0;
    std::memset(&p->h, 0, sizeof(p->h));
    // (a failed create leaves no handle: the destructor's release of a zero handle is a no-op error)
    return fail(RFX_ENOMEM, "hipMemCreate(%zu) failed", bytes);
  }
  return vmm_map(device, {p}, out);
}

int64_t gcd64(int64_t a, int64_t b) { return b ? gcd64(b, a % b) : a; }
int64_t lcm64(int64_t a, int64_t b) { return a / gcd64(a, b) * b; }

struct Index {
  int device = 0;
  int dim = 0;
  int dtype = 0;
  int64_t rows = 0;
  int64_t capacity = 0;
  int64_t live = 0;
  void* data = nullptr;
  // the rows' and the int8 codes' mappings (virtual memory; null with plain hipMalloc buffers); a union view
  // holds its members' physical allocations through its own mappings
  std::shared_ptr<Mapping> rows_map, codes_map;
  bool view = false;         // a union view (rfx_union_create): read-only, owns no physical memory of its own
  int64_t layout_gen = 0;    // bumped whenever data / scodes move (growth, a rebuilt or dropped copy)
  std::vector<int64_t> view_bases;                  // a view: member m's rows start at view_bases[m]
  std::vector<std::weak_ptr<Index>> view_members;   // a view: its members
  std::vector<int64_t> view_gens;                   // a view: the members' layout_gen at creation
  std::vector<uint8_t> tomb;  // host bitmap (1 = deleted), mirrors the NaN rows on device
  std::shared_timed_mutex mu;
  // per-stream launch state of the single-launch VALU search (zeroed once, left zero by every
  // launch); keyed by stream so concurrent searches on different streams never share it
  std::mutex state_mu;
  std::map<hipStream_t, uint32_t*> fused_state;
  // int8 copy of the store for the exact two-pass scan (k_screen.hip): codes
  // [scap][dim], per 32-row tile a 16-B record (scale, live word), and stats[3] (max row norm, max
  // quantisation-error norm, max tile scale; f32 bits).  screen: 0 off, 1 on, 2 on with every batch sent to the
  // exact fallback (tests of the fallback path).
  int screen = 0;
  int screen_dropped = 0;  // an append outgrew what the copy could follow: dropped, the index is exact
  int64_t scap = 0;
  int8_t* scodes = nullptr;
  void* smeta = nullptr;  // per tile {f32 scale, u32 live word, 0, 0}
  uint32_t* sstats = nullptr;
  int64_t row_bytes() const { return (int64_t)dim * esize(dtype); }
};

void screen_free(Index& ix) {
  if (ix.codes_map || ix.scodes) ++ix.layout_gen;
  if (ix.codes_map) {
    (void)hipDeviceSynchronize();  // no search still reads the codes: then unmap
    ix.codes_map.reset();
  } else if (ix.scodes) {
    (void)hipFree(ix.scodes);
  }
  for (void* p : {ix.smeta, (void*)ix.sstats})
    if (p) (void)hipFree(p);
  ix.scodes = nullptr;
  ix.smeta = nullptr;
  ix.sstats = nullptr;
  ix.scap = 0;
}

int64_t env_bytes(const char* name, int64_t dflt) {
  const char* e = getenv(name);  // read at every build: tests and services may change it
  return e && *e ? atoll(e) : dflt;
}

// Device bytes of the int8 copy for `cap` rows: codes, tile records, stats.
int64_t screen_bytes(int64_t cap, int dim) { return cap * dim + cap / 32 * 16 + 256; }

// Does a copy of `cap` rows fit?  Under RFX_SCREEN_MAX_BYTES (when set) and in the device's free memory
// minus RFX_SCREEN_RESERVE_BYTES (default 4 GiB: search workspaces, the next growth of the rows).
int screen_fits(const Index& ix, int64_t cap) {
  const int64_t need = screen_bytes(cap, ix.dim) - (ix.scodes ? screen_bytes(ix.scap, ix.dim) : 0);
  const int64_t cap_bytes = env_bytes("RFX_SCREEN_MAX_BYTES", -1);
  if (cap_bytes >= 0 && screen_bytes(cap, ix.dim) > cap_bytes)
    return fail(RFX_ECAPACITY, "int8 copy of %lld rows needs %lld B > RFX_SCREEN_MAX_BYTES %lld", (long long)cap,
                (long long)screen_bytes(cap, ix.dim), (long long)cap_bytes);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return fail(RFX_EDEVICE, "hipMemGetInfo failed");
  const int64_t reserve = env_bytes("RFX_SCREEN_RESERVE_BYTES", (int64_t)4 << 30);
  if (need + reserve > (int64_t)free_b)
    return fail(RFX_ECAPACITY, "int8 copy of %lld rows needs %lld B more; the device has %zu B free (reserve %lld B)",
                (long long)cap, (long long)need, free_b, (long long)reserve);
  return RFX_OK;
}

// (Re)build the whole int8 copy for the current capacity.
int screen_build(Index& ix, hipStream_t st) {
  const int64_t cap = ix.capacity, nt = cap / 32;
  if (cap > 0) {
    const int rc = screen_fits(ix, cap);
    if (rc) return rc;
  }
  screen_free(ix);
  if (cap == 0) return RFX_OK;
  bool codes_ok;
  if (ix.rows_map) {  // the codes in virtual memory too (capacity_align: cap * dim is a whole number of granules)
    codes_ok = vmm_alloc(ix.device, (size_t)cap * ix.dim, ix.codes_map) == RFX_OK;
    ix.scodes = codes_ok ? (int8_t*)ix.codes_map->va : nullptr;
  } else {
    codes_ok = hipMalloc(&ix.scodes, (size_t)cap * ix.dim) == hipSuccess;
  }
  if (!codes_ok || hipMalloc(&ix.smeta, (size_t)nt * 16) != hipSuccess || hipMalloc(&ix.sstats, 256) != hipSuccess) {
    screen_free(ix);
    return fail(RFX_ECAPACITY, "hipMalloc failed for the int8 screen copy (%lld rows)", (long long)cap);
  }
  ix.scap = cap;
  RFX_HIP(hipMemsetAsync(ix.scodes, 0, (size_t)cap * ix.dim, st));
  RFX_HIP(hipMemsetAsync(ix.smeta, 0, (size_t)nt * 16, st));
  RFX_HIP(hipMemsetAsync(ix.sstats, 0, 256, st));
  rfx::launch_screen_quantize(ix.data, ix.dim, ix.dtype, 0, (ix.rows + 31) / 32, nullptr, ix.scodes, ix.smeta, ix.sstats, st);
  RFX_HIP(hipGetLastError());
  RFX_HIP(hipStreamSynchronize(st));
  return RFX_OK;
}

// Keep the int8 copy current after rows [first, rows) were written: re-quantise the tiles they
// touch (the first one may have gained rows, so its scale can change); a grown buffer is rebuilt.
int screen_update(Index& ix, int64_t first, hipStream_t st) {
  if (!ix.screen) return RFX_OK;
  if (ix.scap != ix.capacity) {
    const int rc = screen_build(ix, st);
    if (rc == RFX_ECAPACITY) {  // the rows are written: drop the copy, the index answers exactly
      screen_free(ix);
      ix.screen = 0;
      ix.screen_dropped = 1;
      return RFX_OK;
    }
    return rc;
  }
  const int64_t t0 = first / 32, t1 = (ix.rows + 31) / 32;
  if (t1 > t0) {
    rfx::launch_screen_quantize(ix.data, ix.dim, ix.dtype, t0, t1 - t0, nullptr, ix.scodes, ix.smeta, ix.sstats, st);
    RFX_HIP(hipGetLastError());
    RFX_HIP(hipStreamSynchronize(st));
  }
  return RFX_OK;
}

// The caller holds ix.state_mu (`slk`) from this lookup until its launches on `st` are enqueued: the
// reset below frees every state after a device-wide drain, and a state handed out but not yet used by
// an enqueued launch would otherwise be freed under its holder.  Once enqueued, the drain
// waits for the launch, which leaves its state zero.
int fused_state(Index& ix, hipStream_t st, uint32_t** out, const std::unique_lock<std::mutex>& slk) {
  if (!slk.owns_lock() || slk.mutex() != &ix.state_mu) return fail(RFX_EINVAL, "search state lock not held");
  auto it = ix.fused_state.find(st);
  if (it != ix.fused_state.end()) {
    *out = it->second;
    return RFX_OK;
  }
  // bounded: callers that make a stream per request would grow the map forever.  Past 64
  // streams every launch is drained (a launch leaves its state zeroed when it completes), then all
  // states are freed; the streams that search again get fresh ones.
  if (ix.fused_state.size() >= 64) {
    RFX_HIP(hipDeviceSynchronize());
    for (auto& kv : ix.fused_state) RFX_HIP(hipFree(kv.second));
    ix.fused_state.clear();
  }
  uint32_t* p = nullptr;
  const size_t bytes = (size_t)rfx::kValuFusedStateWords * 4;
  if (hipMalloc(&p, bytes) != hipSuccess) return fail(RFX_ENOMEM, "hipMalloc(%zu) failed (search state)", bytes);
  // zeroed on the stream that will use it: hipMemset is asynchronous to the host and runs on the null
  // stream, which a non-blocking stream does not wait for (round 5: a first search on a fresh torch
  // stream could read the state before it was zeroed)
  RFX_HIP(hipMemsetAsync(p, 0, bytes, st));
  ix.fused_state[st] = p;
  *out = p;
  return RFX_OK;
}

bool fused_enabled() {  // RFX_VALU_FUSED=0: the three-launch path (widen, scan, merge), for A/B runs
  static const bool on = [] {
    const char* e = getenv("RFX_VALU_FUSED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Bounded lock waits: a writer stuck behind long searches (or the reverse) gets RFX_EBUSY, which
// the host maps to a TimeoutError so the reference's retry paths apply (gemini_rag.py:17-27,
// ingestion.py:35-52).  RFX_LOCK_TIMEOUT_MS, default 30 s.
std::chrono::milliseconds lock_timeout() {
  static const long ms = [] {
    const char* e = getenv("RFX_LOCK_TIMEOUT_MS");
    return e && *e ? atol(e) : 30000L;
  }();
  return std::chrono::milliseconds(ms);
}
#define RFX_WLOCK(ix)                                                                            \
  std::unique_lock<std::shared_timed_mutex> lk((ix)->mu, std::defer_lock);                        \
  if (!lk.try_lock_for(lock_timeout())) return fail(RFX_EBUSY, "index busy: writer lock timed out"); \
  if ((ix)->view) return fail(RFX_EINVAL, "a union view is read-only (write to its member stores)")
#define RFX_RLOCK(ix)                                                                            \
  std::shared_lock<std::shared_timed_mutex> lk((ix)->mu, std::defer_lock);                        \
  if (!lk.try_lock_for(lock_timeout())) return fail(RFX_EBUSY, "index busy: reader lock timed out")

std::mutex g_reg_mu;
std::map<uint64_t, std::shared_ptr<Index>> g_reg;
std::atomic<uint64_t> g_next{1};

std::shared_ptr<Index> get(rfx_index_t h) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(h);
  return it == g_reg.end() ? nullptr : it->second;
}

// Invariant: rows [rows, capacity) of the device buffer hold NaN, so a scan tile that runs past
// the last row (capacity is a multiple of 128 rows) reads rows that can never be ranked.
int fill_tail_nan(Index& ix, hipStream_t st) {
  const int64_t n = ix.capacity - ix.rows;
  if (n <= 0) return RFX_OK;
  const uint32_t pattern = ix.dtype == RFX_F32 ? 0x7fc00000u : (ix.dtype == RFX_BF16 ? 0x7fc07fc0u : 0x7e007e00u);
  RFX_HIP(hipMemsetD32Async((hipDeviceptr_t)((uint8_t*)ix.data + ix.rows * ix.row_bytes()), (int)pattern,
                            (size_t)(n * ix.row_bytes() / 4), st));
  RFX_HIP(hipStreamSynchronize(st));
  return RFX_OK;
}

// Capacity granule (rows): whole 128-row scan tiles; with virtual memory also a whole number of granules of
// the rows' bytes AND of the int8 copy's (d bytes per row), so members of a union view map back to back at
// row bases that are multiples of 128 (8,192 rows at d 768 with a 2-MiB granule).
int64_t capacity_align(const Index& ix) {
  const int64_t g = (int64_t)vmm_granularity(ix.device);
  if (!g) return 128;
  return lcm64(lcm64(128, g / gcd64(g, ix.row_bytes())), g / gcd64(g, (int64_t)ix.dim));
}

int grow(Index& ix, int64_t need, hipStream_t st) {
  if (need <= ix.capacity) return RFX_OK;
  int64_t cap = ix.capacity > 0 ? ix.capacity : 1024;
  while (cap < need) cap = cap + cap / 2 + 1024;
  const int64_t al = capacity_align(ix);
  cap = (cap + al - 1) / al * al;
  void* p = nullptr;
  std::shared_ptr<Mapping> m;
  const size_t bytes = (size_t)cap * ix.row_bytes();
  if (vmm_granularity(ix.device)) {
    const int rc = vmm_alloc(ix.device, bytes, m);
    if (rc) return fail(RFX_ENOMEM, "device memory for %lld rows: %s", (long long)cap, g_err.c_str());
    p = m->va;
  } else if (hipMalloc(&p, bytes) != hipSuccess) {
    return fail(RFX_ENOMEM, "hipMalloc(%zu) failed for index", bytes);
  }
  if (ix.rows > 0) {
    RFX_HIP(hipMemcpyAsync(p, ix.data, (size_t)ix.rows * ix.row_bytes(), hipMemcpyDeviceToDevice, st));
    RFX_HIP(hipStreamSynchronize(st));
  }
  if (ix.rows_map) {
    RFX_HIP(hipDeviceSynchronize());  // no search still reads the old rows: then unmap
    ix.rows_map.reset();
  } else if (ix.data) {
    RFX_HIP(hipFree(ix.data));  // hipFree waits for in-flight work on the old buffer
  }
  ix.rows_map = m;
  ix.data = p;
  ix.capacity = cap;
  ++ix.layout_gen;
  return fill_tail_nan(ix, st);
}

// ---- search workspace layout ------------------------------------------------------------------
struct SearchLayout {
  int kernel;        // 0 VALU (nq <= 8); 1 MFMA 128×BN (nq <= 64); 2 MFMA 256×256; 3 query-stationary MFMA;
                     // 6 config-3 kernel (d 768); 7 / 8 d-1024 kernels (config 4); 9 f32 stores
  rfx::ValuPlan vp;
  rfx::MfmaPlan mp;
  int64_t n_cand;    // candidates per query
  size_t q_off, q_bytes, tau_off, cs_off, cr_off, total;
  // kernel 10 (the two-pass scan): the exact plan above (kernel fbk, regions q/tau/cs/cr) is its
  // gated fallback; the screen's own regions follow it
  int fbk;
  rfx::MfmaPlan sp;
  size_t s_tau, s_cs, s_cr, s_drop, s_qc, s_qe2, s_gate, s_diag;
  // the one-launch VALU searches (kernel 11, the fused exact search) write (score, row) pairs: for a
  // records / row-offset output they go here first and one pack launch converts them (sharded stores)
  size_t pk_off, pk_r_off;
  // kernel 11 (nq <= 8 on a VALU plan): the exact score keys of the record entries its blocks re-score
  // before they arrive ([nq][blocks][16] u32, beside the records at cs_off / cr_off)
  size_t cx_off;
};

size_t align_up(size_t x) { return (x + 255) / 256 * 256; }

int make_layout(const Index& ix, int64_t nq, int k, SearchLayout& L, bool search = false, int scan_blocks = 0);

// The search plan: the exact layout, extended by the two-pass scan's regions when the index holds an
// int8 copy and the exact plan is the config-3 / config-4 kernel (6 / 8) it falls back to.
int make_search_layout(const Index& ix, int64_t nq, int k, SearchLayout& L, int scan_blocks = 0) {
  return make_layout(ix, nq, k, L, true, scan_blocks);
}

int make_layout(const Index& ix, int64_t nq, int k, SearchLayout& L, bool search, int scan_blocks) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0) return fail(RFX_EINVAL, "nq < 0");
  if (ix.rows >= (int64_t)INT32_MAX) return fail(RFX_EUNSUPPORTED, "shard exceeds 2^31-1 rows");
  L = SearchLayout{};
  L.vp = rfx::plan_scan_valu(ix.rows, ix.dim, ix.dtype, nq, k);
  L.kernel = 0;
  // With an int8 copy every batch of nq > 8 (k <= 10) takes the two-pass scan (kernel 10: the 8-wave kernel
  // for nq > 64, the 2-wave one for 9..64), whose gated fallback is the exact scan planned here: kernel 6
  // (bf16 / f16, d 768), 8 (d 1024) or 9 (f32, d 768) whatever nq, padded to their query groups.
  const bool two_pass = search && ix.screen && ix.rows > 0 && k <= 10 && rfx::screen_supported(ix.dim, ix.dtype);
  if (nq > 8) {
    if (nq > 128 || (two_pass && nq > 8)) {
      L.mp = rfx::plan_scan_mfma6(ix.rows, ix.dim, ix.dtype, nq, k);
      if (L.mp.ok) L.kernel = 6;
    }
    if (L.kernel == 0 && (nq > 64 || two_pass)) {  // d = 1024: kernel 8 (k-split wave pairs)
      L.mp = rfx::plan_scan_mfma8(ix.rows, ix.dim, ix.dtype, nq, k);
      if (L.mp.ok) L.kernel = 8;
    }
    if (L.kernel == 0 && nq > 64) {
      L.mp = rfx::plan_scan_mfma3(ix.rows, ix.dim, ix.dtype, nq, k);
      if (L.mp.ok) L.kernel = 3;
    }
    if (L.kernel == 0 && ix.dtype == RFX_F32) {
      // (kernel 9 plans nq > 16; as the two-pass scan's fallback it also takes 9..16 questions, padded to 128)
      L.mp = rfx::plan_scan_mfma9(ix.rows, ix.dim, ix.dtype, two_pass ? std::max<int64_t>(nq, 17) : nq, k);
      if (L.mp.ok) L.kernel = 9;
    }
    if (L.kernel == 0 && nq > 128) {
      L.mp = rfx::plan_scan_mfma2(ix.rows, ix.dim, ix.dtype, nq, k);
      if (L.mp.ok) L.kernel = 2;
    }
    if (L.kernel == 0) {
      L.mp = rfx::plan_scan_mfma(ix.rows, ix.dim, ix.dtype, nq, k);
      if (L.mp.ok) L.kernel = 1;
    }
  }
  size_t tau_bytes = 0;
  if (L.kernel) {
    L.n_cand = L.mp.n_lists * L.mp.k_lane;
    L.q_bytes = (size_t)L.mp.nq_pad * ix.dim * (L.kernel == 9 ? 4 : 2);
    if (L.kernel == 6)  // (the debug build's kernel-5 ablations use the same [nq_pad][16] table)
      tau_bytes = rfx::tau_bytes_mfma6(L.mp);
    else if (L.kernel == 8)
      tau_bytes = rfx::tau_bytes_mfma8(L.mp);
    else if (L.kernel == 9)
      tau_bytes = rfx::tau_bytes_mfma9(L.mp);
    else if (L.kernel >= 2)
      tau_bytes = (size_t)(L.mp.nq_pad + 256) * 4;  // + slack: 1 KB threshold DMA per group
  } else {
    if (!L.vp.ok) return fail(RFX_EUNSUPPORTED, "no scan kernel for dim=%d dtype=%d k=%d", ix.dim, ix.dtype, k);
    L.n_cand = (int64_t)L.vp.n_lists * L.vp.k_slot;
    L.q_bytes = (size_t)nq * ix.dim * 4;
    tau_bytes = (size_t)nq * 4;  // per-query pruning bounds of the VALU scan
  }
  if (ix.rows == 0) L.n_cand = 0;
  L.q_off = 0;
  L.tau_off = align_up(L.q_bytes);
  L.cs_off = L.tau_off + align_up(tau_bytes);
  L.cr_off = L.cs_off + align_up((size_t)nq * L.n_cand * 4);
  L.total = L.cr_off + align_up((size_t)nq * L.n_cand * 4);
  L.fbk = 0;
  if (search && ix.screen && ix.rows > 0 && (L.kernel == 6 || L.kernel == 8 || L.kernel == 9)) {
    L.sp = rfx::plan_scan_screen(ix.rows, ix.dim, ix.dtype, nq, k, scan_blocks);
    // the regions are sized (and placed) by the default plan, the most workgroups and lists any
    // scan_blocks gives: every offset, the gate and diag words included, is then the same whatever
    // scan_blocks a search used (rfx_screen_diag and rfx_search_plan build the default layout)
    const rfx::MfmaPlan smax = scan_blocks ? rfx::plan_scan_screen(ix.rows, ix.dim, ix.dtype, nq, k, 0) : L.sp;
    if (L.sp.ok && smax.ok) {
      L.fbk = L.kernel;
      L.kernel = 10;
      const size_t nc = (size_t)std::max(L.sp.n_lists, smax.n_lists) * std::max(L.sp.k_lane, smax.k_lane);
      L.s_tau = L.total;
      L.s_cs = L.s_tau + align_up(std::max(rfx::tau_bytes_screen(L.sp), rfx::tau_bytes_screen(smax)));
      L.s_cr = L.s_cs + align_up((size_t)nq * nc * 4);
      L.s_drop = L.s_cr + align_up((size_t)nq * nc * 4);
      L.s_qc = L.s_drop + align_up((size_t)nq * std::max(L.sp.n_lists, smax.n_lists) * 4);
      L.s_qe2 = L.s_qc + align_up((size_t)L.sp.nq_pad * ix.dim);
      L.s_gate = L.s_qe2 + align_up((size_t)L.sp.nq_pad * 4);
      L.s_diag = L.s_gate + 256;
      L.total = L.s_diag + align_up((size_t)nq * 8);
    }
  }
  L.pk_off = L.pk_r_off = 0;
  if (search && L.kernel == 0 && nq > 0) {
    L.pk_off = L.total;
    L.pk_r_off = L.pk_off + align_up((size_t)nq * k * 4);
    L.total = L.pk_r_off + align_up((size_t)nq * k * 8);
  }
  L.cx_off = 0;
  if (search && L.kernel == 0 && nq >= 1 && nq <= 8 && ix.rows > 0) {
    // (whether or not the index holds an int8 copy yet: a workspace sized before enable_screen fits)
    L.cx_off = L.total;
    L.total = L.cx_off + align_up((size_t)nq * L.n_cand * 4);
  }
  return RFX_OK;
}

// query staging and thresholds live in the front of ws (q_off, tau_off < cs_off)
size_t scan_ws_bytes(const SearchLayout& L) { return L.cs_off; }

// ---- append-only row files (rfx/store.py) ----------------------------------------------------------
constexpr int64_t kRowsHdr = 64;

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

bool full_write(int fd, const uint8_t* p, size_t n) {
  while (n) {
    const ssize_t w = write(fd, p, n);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool full_pread(int fd, uint8_t* p, size_t n, off_t off) {
  while (n) {
    const ssize_t r = pread(fd, p, n, off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    off += r;
    n -= (size_t)r;
  }
  return true;
}

void rows_header(const Index& ix, uint8_t hdr[kRowsHdr]) {
  memset(hdr, 0, kRowsHdr);
  memcpy(hdr, "RFXROWS1", 8);
  const uint32_t v[3] = {1u, (uint32_t)ix.dim, (uint32_t)ix.dtype};
  memcpy(hdr + 8, v, sizeof(v));
}

// pinned staging buffers for file <-> device copies
struct Pinned {
  void* p = nullptr;
  explicit Pinned(size_t n) {
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) p = nullptr;
  }
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
};
constexpr size_t kStage = (size_t)64 << 20;

// mask: optional row mask on the device (metadata filter), (rows + 31) / 32 words, checked by the
// caller; every production scan kernel applies it in its epilogue.
int scan_into(Index& ix, const SearchLayout& L, const void* queries, int64_t nq, float* cs, int32_t* cr,
              uint8_t* ws, hipStream_t st, const uint32_t* mask = nullptr) {
  if (ix.rows == 0 || nq == 0) return RFX_OK;
  if (L.kernel >= 1) {
    // the MFMA scans read queries as [nq_pad][dim]: a batch that is already a whole number of
    // query groups (config 3: 256) is read in place, with no padding launch
    const void* qpad = queries;
    if (nq != L.mp.nq_pad || ((uintptr_t)queries & 15)) {
      qpad = ws + L.q_off;
      rfx::launch_pad_queries(queries, nq, L.mp.nq_pad, ix.dim, L.kernel == 9 ? 4 : 2, (void*)qpad, st);
    }
    uint32_t* tau = (uint32_t*)(ws + L.tau_off);
    const int rc =
        L.kernel == 6 ? rfx::launch_scan_mfma6(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs, cr, st, mask)
        : L.kernel == 8 ? rfx::launch_scan_mfma8(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs, cr, st, mask)
        : L.kernel == 9 ? rfx::launch_scan_mfma9(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs, cr, st, mask)
        : L.kernel == 3 ? rfx::launch_scan_mfma3(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs, cr, st, mask)
        : L.kernel == 2 ? rfx::launch_scan_mfma2(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs, cr, st, mask)
                        : rfx::launch_scan_mfma(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, cs, cr, st, mask);
    if (rc != 0) return fail(RFX_EUNSUPPORTED, "MFMA scan launch rejected (%d)", rc);
  } else {
    float* qf = (float*)(ws + L.q_off);
    uint32_t* tau = (uint32_t*)(ws + L.tau_off);
    rfx::launch_widen_queries(queries, nq * ix.dim, ix.dtype, qf, st, tau, nq);
    if (rfx::launch_scan_valu(L.vp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qf, (int)nq, cs, cr, st, mask, tau) != 0)
      return fail(RFX_EUNSUPPORTED, "VALU scan launch rejected");
  }
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

// The exact two-pass scan (kernel 10 + k_screen.hip): query codes, int8 screen,
// select (survivors -> exact re-score -> top-k); then the exact scan + merge of the fallback plan,
// gated on the device word the select kernel sets when a query's survivors may be incomplete.
// Writes (out_s, out_r) or, with out_rec, the {score, pad, row + row_offset} records.
int screen_search(Index& ix, const SearchLayout& L, const void* queries, int64_t nq, int k, const uint32_t* mask,
                  int64_t row_offset, float* out_s, int64_t* out_r, void* out_rec, uint8_t* ws, hipStream_t st,
                  void* ev0 = nullptr, void* ev1 = nullptr, int stages = 3) {
  if (nq == 0) return RFX_OK;
  int8_t* qc = (int8_t*)(ws + L.s_qc);
  float* qe2 = (float*)(ws + L.s_qe2);
  uint32_t* stau = (uint32_t*)(ws + L.s_tau);
  float* scs = (float*)(ws + L.s_cs);
  int* scr = (int*)(ws + L.s_cr);
  uint32_t* drops = (uint32_t*)(ws + L.s_drop);
  uint32_t* gate = (uint32_t*)(ws + L.s_gate);
  int* diag = (int*)(ws + L.s_diag);
  uint32_t* tau = (uint32_t*)(ws + L.tau_off);
  // the fallback's threshold table ([its nq_pad][16]) is zeroed by the query quantiser: no memset launch
  if (stages & 1) {
    rfx::ScreenSeed sd;
    sd.X8 = ix.scodes;
    sd.tmeta = ix.smeta;
    sd.nrows = (int)ix.rows;
    sd.mask = mask;
    sd.kl = L.sp.k_lane;
    rfx::launch_screen_queries(queries, ix.dtype, ix.dim, nq, L.sp.nq_pad, qc, qe2, ix.sstats, stau, gate, tau,
                               L.mp.nq_pad, st, &sd);
    if (ev0) RFX_HIP(hipEventRecord((hipEvent_t)ev0, st));
    if (rfx::launch_scan_screen(L.sp, ix.scodes, ix.smeta, ix.sstats, (int)ix.rows, ix.dim, qc, qe2, (int)nq, stau, scs,
                                scr, drops, st, mask) != 0)
      return fail(RFX_EUNSUPPORTED, "screen scan launch rejected");
    if (ev1) RFX_HIP(hipEventRecord((hipEvent_t)ev1, st));
  }
  if (!(stages & 2)) {
    RFX_HIP(hipGetLastError());
    return RFX_OK;
  }
  // the select and the gated exact pass read the queries with 16-B loads: an unaligned batch (or one
  // that is not a whole number of the fallback's query groups) is copied once into the workspace
  const void* qpad = queries;
  if (nq != L.mp.nq_pad || ((uintptr_t)queries & 15)) {
    qpad = ws + L.q_off;
    rfx::launch_pad_queries(queries, nq, L.mp.nq_pad, ix.dim, esize(ix.dtype), (void*)qpad, st);
  }
  float* cs = (float*)(ws + L.cs_off);
  int32_t* cr = (int32_t*)(ws + L.cr_off);
  if (rfx::launch_screen_select(scs, scr, drops, L.sp.n_lists, L.sp.k_lane, qe2, qpad, ix.data, ix.dim, ix.dtype, nq,
                                k, row_offset, out_s, out_r, out_rec, gate, diag, ix.screen == 2, st) != 0)
    return fail(RFX_EUNSUPPORTED, "screen select k=%d unsupported", k);
  // gated exact pass (no work unless the select kernel set the gate)
  const int rc = L.fbk == 6 ? rfx::launch_scan_mfma6(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs,
                                                     cr, st, mask, gate, true)
                 : L.fbk == 8 ? rfx::launch_scan_mfma8(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs,
                                                       cr, st, mask, gate, true)
                              : rfx::launch_scan_mfma9(L.mp, ix.data, (int)ix.rows, ix.dim, ix.dtype, qpad, (int)nq, tau, cs,
                                                       cr, st, mask, gate, true);
  if (rc != 0) return fail(RFX_EUNSUPPORTED, "fallback scan launch rejected (%d)", rc);
  // (the fallback's final top-k re-scored by the two-pass rule: the same bits as the select's answer)
  const rfx::Rescore rs{ix.data, queries, ix.dim, ix.dtype, ix.rows};
  if (rfx::launch_topk_merge_lists(cs, cr, 0, nq, L.n_cand, L.mp.k_lane, k, row_offset, out_rec ? nullptr : out_s,
                                   out_rec ? nullptr : out_r, out_rec, st, /*sorted=*/true, gate, &rs) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

// RFX_K11_ABLATE (profiling only; wrong results): kernel 11 phase-skip bits 2 (row stream), 4 (query
// quantiser), 8 (last block's select), 16 (its re-score and rank), 32 (its a_k over the records), 64 (the
// waves' list offers)
int k11_ablate() {
  static const int v = [] {
    const char* e = getenv("RFX_K11_ABLATE");
    return e ? (atoi(e) & 126) : 0;
  }();
  return v;
}

// Kernel 11 (k_screen_valu.hip): a few questions (nq <= 8) on an index holding the int8 copy, on a
// VALU plan with lists of 16 (5 <= k <= 16) — one launch, plus the gated exact one-launch search.
// Kernel-11 launches of one device run one at a time once more than one stream issues them: each then
// waits for the device's previous one (an event) when that one went to another stream.  Kernel 11 holds
// one workgroup per CU and its early blocks wait (bounded) for the last one's verdict; two such launches
// side by side can fill the CUs with waiting blocks until the bound ends the waits (correct — the
// in-launch fallback needs no co-residency — but slow).  A device whose kernel-11 launches all come from
// one stream records nothing (an event record per search cost config 2 ~5 us a search, round 5).
struct K11Order {
  std::mutex mu;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  bool used = false;
  bool multi = false;     // a second stream has issued kernel 11 on this device recently
  bool recorded = false;  // ev holds the previous launch
  int same = 0;           // launches in a row from the last stream (kK11OrderDecay of them end `multi`)
};
// after this many kernel-11 launches in a row from one stream the device goes back to recording
// nothing (a process that once searched from two streams does not pay an event per search forever;
// the next second-stream launch re-enables the order, and is correct without it)
constexpr int kK11OrderDecay = 256;
K11Order& k11_order(int device) {
  static K11Order o[64];
  return o[device & 63];
}
// RFX_K11_UNORDERED=1 (tests, read at every search): no ordering — the in-launch fallback's
// correctness without it
bool k11_unordered() {
  const char* e = getenv("RFX_K11_UNORDERED");
  return e && e[0] == '1';
}

bool screen_valu_eligible(const Index& ix, const SearchLayout& L, int64_t nq, int k) {
  return ix.screen && ix.rows > 0 && L.kernel == 0 && L.cx_off && nq >= 1 && nq <= 8 && k <= 16 && L.vp.k_slot == 16 &&
         rfx::screen_supported(ix.dim, ix.dtype) && fused_enabled();
}

}  // namespace

namespace rfx {
int api_fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace rfx

extern "C" {

const char* rfx_last_error(void) { return g_err.c_str(); }

int rfx_version(void) { return 100; }

int rfx_device_count(int* out_n) {
  if (!out_n) return fail(RFX_EINVAL, "null out");
  int n = 0;
  RFX_HIP(hipGetDeviceCount(&n));
  *out_n = n;
  return RFX_OK;
}

int rfx_init(int device) {
  RFX_HIP(hipSetDevice(device));
  return RFX_OK;
}

int rfx_index_create(int device, int dim, int dtype, int64_t capacity, rfx_index_t* out) {
  if (!out) return fail(RFX_EINVAL, "null out");
  if (dim <= 0 || dim % 64 != 0 || dim > 4096) return fail(RFX_EINVAL, "dim=%d must be a positive multiple of 64 <= 4096", dim);
  if (!valid_dtype(dtype)) return fail(RFX_EINVAL, "bad dtype %d", dtype);
  if (capacity < 0) return fail(RFX_EINVAL, "capacity < 0");
  RFX_HIP(hipSetDevice(device));
  auto ix = std::make_shared<Index>();
  ix->device = device;
  ix->dim = dim;
  ix->dtype = dtype;
  if (capacity > 0) {
    int rc = grow(*ix, capacity, nullptr);
    if (rc) return rc;
  }
  const uint64_t h = g_next++;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[h] = ix;
  }
  *out = h;
  return RFX_OK;
}

int rfx_index_destroy(rfx_index_t h) {
  std::shared_ptr<Index> ix;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(h);
    if (it == g_reg.end()) return fail(RFX_EINVAL, "unknown index handle %llu", (unsigned long long)h);
    ix = it->second;
    g_reg.erase(it);
  }
  std::unique_lock<std::shared_timed_mutex> lk(ix->mu);  // waits for in-flight searches: never EBUSY
  RFX_HIP(hipSetDevice(ix->device));
  if (ix->rows_map || ix->view) {
    RFX_HIP(hipDeviceSynchronize());  // no launch still reads the mapped rows: then unmap
    ix->rows_map.reset();
    ix->data = nullptr;
  } else if (ix->data) {
    RFX_HIP(hipFree(ix->data));
    ix->data = nullptr;
  }
  for (auto& kv : ix->fused_state) RFX_HIP(hipFree(kv.second));
  ix->fused_state.clear();
  screen_free(*ix);
  return RFX_OK;
}

// ---- union views (a question over several stores in one launch; gemini_rag.py:463-469) ------------------------
}  // extern "C"
namespace {
__global__ void stats_max_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst) {
  if (threadIdx.x < 3) atomicMax(dst + threadIdx.x, src[threadIdx.x]);  // non-negative f32 bits order as u32
}

// the members of a view, locked shared for the caller's scope; `stale` when one is gone or moved its memory
struct ViewMembers {
  std::vector<std::shared_ptr<Index>> ix;
  std::vector<std::shared_lock<std::shared_timed_mutex>> locks;
  bool stale = false;
};
int lock_members(const Index& v, ViewMembers& vm) {
  for (size_t m = 0; m < v.view_members.size(); ++m) {
    auto ix = v.view_members[m].lock();
    if (!ix) {
      vm.stale = true;
      return RFX_OK;
    }
    std::shared_lock<std::shared_timed_mutex> lk(ix->mu, std::defer_lock);
    if (!lk.try_lock_for(lock_timeout())) return fail(RFX_EBUSY, "union member busy: reader lock timed out");
    if (ix->layout_gen != v.view_gens[m] || (v.screen != 0) != (ix->screen != 0 && ix->scodes != nullptr)) vm.stale = true;
    vm.ix.push_back(ix);
    vm.locks.push_back(std::move(lk));
  }
  return RFX_OK;
}

// the view's own bytes: the members' tile records copied into one table and the max of their stats
int view_refresh(Index& v, const ViewMembers& vm, hipStream_t st) {
  if (!v.screen) return RFX_OK;
  RFX_HIP(hipMemsetAsync(v.sstats, 0, 256, st));
  for (size_t m = 0; m < vm.ix.size(); ++m) {
    const Index& ix = *vm.ix[m];
    RFX_HIP(hipMemcpyAsync((uint8_t*)v.smeta + v.view_bases[m] / 32 * 16, ix.smeta, (size_t)ix.capacity / 32 * 16,
                           hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(stats_max_kernel, dim3(1), dim3(64), 0, st, ix.sstats, v.sstats);
  }
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}
}  // namespace
extern "C" {

int rfx_union_create(const rfx_index_t* members, int n, void* stream, rfx_index_t* out, int64_t* out_bases) {
  if (!members || n < 1 || !out) return fail(RFX_EINVAL, "null members / out, or n < 1");
  auto v = std::make_shared<Index>();
  v->view = true;
  ViewMembers vm;
  for (int m = 0; m < n; ++m) {
    auto ix = get(members[m]);
    if (!ix) return fail(RFX_EINVAL, "unknown index handle (member %d)", m);
    if (ix->view) return fail(RFX_EINVAL, "member %d is itself a union view", m);
    if (m == 0) {
      v->device = ix->device;
      v->dim = ix->dim;
      v->dtype = ix->dtype;
    } else if (ix->device != v->device || ix->dim != v->dim || ix->dtype != v->dtype) {
      return fail(RFX_EINVAL, "member %d differs in device / dim / dtype", m);
    }
    v->view_members.push_back(ix);
  }
  RFX_HIP(hipSetDevice(v->device));
  if (!vmm_granularity(v->device)) return fail(RFX_EUNSUPPORTED, "union views need HIP virtual memory (RFX_VMM=0?)");
  v->view_gens.assign((size_t)n, 0);
  for (int m = 0; m < n; ++m) v->view_gens[m] = v->view_members[m].lock()->layout_gen;
  int rc = lock_members(*v, vm);
  if (rc) return rc;
  if ((int)vm.ix.size() != n) return fail(RFX_EINVAL, "a member was destroyed meanwhile");
  bool screened = true;
  std::vector<std::shared_ptr<Phys>> rows_parts, code_parts;
  for (int m = 0; m < n; ++m) {
    const Index& ix = *vm.ix[m];
    if (!ix.rows_map || ix.capacity == 0)
      return fail(RFX_EUNSUPPORTED, "member %d has no mapped rows (empty, or made without virtual memory)", m);
    v->view_bases.push_back(v->capacity);
    v->capacity += ix.capacity;
    v->live += ix.live;
    rows_parts.insert(rows_parts.end(), ix.rows_map->parts.begin(), ix.rows_map->parts.end());
    screened = screened && ix.screen && ix.codes_map && ix.scap == ix.capacity;
    if (screened) code_parts.insert(code_parts.end(), ix.codes_map->parts.begin(), ix.codes_map->parts.end());
  }
  if ((rc = vmm_map(v->device, rows_parts, v->rows_map))) return rc;
  v->data = v->rows_map->va;
  v->rows = v->capacity;
  v->tomb.assign((size_t)(v->rows + 7) / 8, 0);
  if (screened) {
    if ((rc = vmm_map(v->device, code_parts, v->codes_map))) return rc;
    v->scodes = (int8_t*)v->codes_map->va;
    v->scap = v->capacity;
    if (hipMalloc(&v->smeta, (size_t)v->capacity / 32 * 16) != hipSuccess || hipMalloc(&v->sstats, 256) != hipSuccess) {
      screen_free(*v);
      return fail(RFX_ENOMEM, "hipMalloc failed for the view's tile records");
    }
    v->screen = 1;
    if ((rc = view_refresh(*v, vm, (hipStream_t)stream))) return rc;
  }
  for (auto& ix : vm.ix)
    if (ix->screen_dropped) v->screen_dropped = 1;
  if (out_bases)
    for (int m = 0; m < n; ++m) out_bases[m] = v->view_bases[m];
  const uint64_t h = g_next++;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[h] = v;
  }
  *out = h;
  return RFX_OK;
}

int rfx_union_refresh(rfx_index_t view, void* stream, int* out_stale) {
  auto v = get(view);
  if (!v || !out_stale) return fail(RFX_EINVAL, "unknown view handle / null out");
  if (!v->view) return fail(RFX_EINVAL, "not a union view");
  std::unique_lock<std::shared_timed_mutex> lk(v->mu, std::defer_lock);  // (searches of the view read the records)
  if (!lk.try_lock_for(lock_timeout())) return fail(RFX_EBUSY, "view busy: lock timed out");
  RFX_HIP(hipSetDevice(v->device));
  ViewMembers vm;
  int rc = lock_members(*v, vm);
  if (rc) return rc;
  *out_stale = vm.stale ? 1 : 0;
  return vm.stale ? RFX_OK : view_refresh(*v, vm, (hipStream_t)stream);
}

int rfx_index_info(rfx_index_t h, int* dim, int* dtype, int64_t* rows, int64_t* capacity, int64_t* live_rows) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  if (dim) *dim = ix->dim;
  if (dtype) *dtype = ix->dtype;
  if (rows) *rows = ix->rows;
  if (capacity) *capacity = ix->capacity;
  if (live_rows) *live_rows = ix->live;
  return RFX_OK;
}

int rfx_index_reserve(rfx_index_t h, int64_t capacity) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_WLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  const int rc = grow(*ix, capacity, nullptr);
  return rc ? rc : screen_update(*ix, ix->rows, nullptr);
}

int rfx_index_add(rfx_index_t h, const void* vecs, int64_t n, int src_is_device, int64_t* out_first_row, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (n < 0 || (n > 0 && !vecs)) return fail(RFX_EINVAL, "bad vectors");
  hipStream_t st = (hipStream_t)stream;
  RFX_WLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  int rc = grow(*ix, ix->rows + n, st);
  if (rc) return rc;
  const int64_t first = ix->rows;
  if (n > 0) {
    RFX_HIP(hipMemcpyAsync((uint8_t*)ix->data + first * ix->row_bytes(), vecs, (size_t)n * ix->row_bytes(),
                           src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    if (!src_is_device) RFX_HIP(hipStreamSynchronize(st));  // host buffer may be freed on return
  }
  ix->rows += n;
  ix->live += n;
  ix->tomb.resize((size_t)(ix->rows + 7) / 8, 0);
  if (out_first_row) *out_first_row = first;
  return screen_update(*ix, first, st);
}

int rfx_index_write(rfx_index_t h, int64_t row0, const void* vecs, int64_t n, int src_is_device, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (n < 0 || (n > 0 && !vecs)) return fail(RFX_EINVAL, "bad vectors");
  hipStream_t st = (hipStream_t)stream;
  RFX_WLOCK(ix);
  if (row0 < 0 || row0 + n > ix->rows)
    return fail(RFX_EINVAL, "rows [%lld, %lld) are not rows of the index (%lld)", (long long)row0, (long long)(row0 + n),
                (long long)ix->rows);
  if (n == 0) return RFX_OK;
  RFX_HIP(hipSetDevice(ix->device));
  RFX_HIP(hipMemcpyAsync((uint8_t*)ix->data + row0 * ix->row_bytes(), vecs, (size_t)n * ix->row_bytes(),
                         src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
  for (int64_t r = row0; r < row0 + n; ++r) {  // rewritten rows are live again
    uint8_t& b = ix->tomb[(size_t)(r >> 3)];
    if (b & (1u << (r & 7))) {
      b &= (uint8_t) ~(1u << (r & 7));
      ++ix->live;
    }
  }
  if (ix->screen) {  // re-quantise the tiles the rows touch (their scales and live words change)
    const int64_t t0 = row0 / 32, t1 = (row0 + n + 31) / 32;
    rfx::launch_screen_quantize(ix->data, ix->dim, ix->dtype, t0, t1 - t0, nullptr, ix->scodes, ix->smeta, ix->sstats, st);
    RFX_HIP(hipGetLastError());
  }
  RFX_HIP(hipStreamSynchronize(st));
  return RFX_OK;
}

int rfx_index_add_synthetic(rfx_index_t h, uint64_t seed, int64_t gen_row0, int64_t n, int64_t* out_first_row,
                            void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (n < 0) return fail(RFX_EINVAL, "n < 0");
  hipStream_t st = (hipStream_t)stream;
  RFX_WLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  int rc = grow(*ix, ix->rows + n, st);
  if (rc) return rc;
  const int64_t first = ix->rows;
  if (n > 0) {
    rfx::launch_synth_rows(seed, gen_row0 < 0 ? first : gen_row0, n, ix->dim, ix->dtype,
                           (uint8_t*)ix->data + first * ix->row_bytes(), st);
    RFX_HIP(hipGetLastError());
  }
  ix->rows += n;
  ix->live += n;
  ix->tomb.resize((size_t)(ix->rows + 7) / 8, 0);
  if (out_first_row) *out_first_row = first;
  return screen_update(*ix, first, st);
}

int rfx_index_tombstone(rfx_index_t h, const int64_t* rows_h, int64_t n, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (n < 0 || (n > 0 && !rows_h)) return fail(RFX_EINVAL, "bad rows");
  hipStream_t st = (hipStream_t)stream;
  RFX_WLOCK(ix);
  std::vector<int64_t> todo;
  todo.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = rows_h[i];
    if (r < 0 || r >= ix->rows) return fail(RFX_EINVAL, "row %lld out of range", (long long)r);
    uint8_t& b = ix->tomb[(size_t)r >> 3];
    if (!(b & (1u << (r & 7)))) {
      b |= (uint8_t)(1u << (r & 7));
      todo.push_back(r);
    }
  }
  if (todo.empty()) return RFX_OK;
  RFX_HIP(hipSetDevice(ix->device));
  int64_t* d = nullptr;
  RFX_HIP(hipMalloc(&d, todo.size() * sizeof(int64_t)));
  RFX_HIP(hipMemcpyAsync(d, todo.data(), todo.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
  rfx::launch_nan_rows(ix->data, d, (int64_t)todo.size(), ix->row_bytes(), ix->dtype, st);
  RFX_HIP(hipGetLastError());
  RFX_HIP(hipStreamSynchronize(st));
  RFX_HIP(hipFree(d));
  ix->live -= (int64_t)todo.size();
  if (ix->screen) {  // the tombstoned rows' tiles: code 0, live bit clear, scale over the rest
    if (ix->scap != ix->capacity) return screen_build(*ix, st);
    std::vector<int64_t> tiles;
    for (int64_t r : todo) tiles.push_back(r / 32);
    std::sort(tiles.begin(), tiles.end());
    tiles.erase(std::unique(tiles.begin(), tiles.end()), tiles.end());
    int64_t* td = nullptr;
    RFX_HIP(hipMalloc(&td, tiles.size() * sizeof(int64_t)));
    RFX_HIP(hipMemcpyAsync(td, tiles.data(), tiles.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
    rfx::launch_screen_quantize(ix->data, ix->dim, ix->dtype, 0, (int64_t)tiles.size(), td, ix->scodes, ix->smeta,
                                ix->sstats, st);
    RFX_HIP(hipGetLastError());
    RFX_HIP(hipStreamSynchronize(st));
    RFX_HIP(hipFree(td));
  }
  return RFX_OK;
}

int rfx_index_read(rfx_index_t h, int64_t row0, int64_t n, void* dst, int dst_is_device, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  if (row0 < 0 || n < 0 || row0 + n > ix->rows) return fail(RFX_EINVAL, "rows [%lld, %lld) out of range", (long long)row0, (long long)(row0 + n));
  if (n == 0) return RFX_OK;
  if (!dst) return fail(RFX_EINVAL, "null destination");
  RFX_HIP(hipSetDevice(ix->device));
  hipStream_t st = (hipStream_t)stream;
  RFX_HIP(hipMemcpyAsync(dst, (uint8_t*)ix->data + row0 * ix->row_bytes(), (size_t)n * ix->row_bytes(),
                         dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
  if (!dst_is_device) RFX_HIP(hipStreamSynchronize(st));
  return RFX_OK;
}

int rfx_index_data(rfx_index_t h, void** out_ptr) {
  auto ix = get(h);
  if (!ix || !out_ptr) return fail(RFX_EINVAL, "unknown index handle / null out");
  *out_ptr = ix->data;
  return RFX_OK;
}

// File format (little endian): "RFXIDX01" | u32 version=1 | u32 dim | u32 dtype | u32 0 |
// i64 rows | i64 live | tombstone bitmap ceil(rows/8) B | rows*dim*esize B of row data.
int rfx_index_save(rfx_index_t h, const char* path) {
  auto ix = get(h);
  if (!ix || !path) return fail(RFX_EINVAL, "unknown index handle / null path");
  RFX_RLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return fail(RFX_EIO, "cannot open %s", tmp.c_str());
  const uint32_t hdr[4] = {1u, (uint32_t)ix->dim, (uint32_t)ix->dtype, 0u};
  const int64_t cnt[2] = {ix->rows, ix->live};
  bool ok = fwrite("RFXIDX01", 1, 8, f) == 8 && fwrite(hdr, 4, 4, f) == 4 && fwrite(cnt, 8, 2, f) == 2;
  const size_t tb = (size_t)(ix->rows + 7) / 8;
  if (ok && tb) ok = fwrite(ix->tomb.data(), 1, tb, f) == tb;
  const size_t total = (size_t)ix->rows * ix->row_bytes();
  std::vector<uint8_t> buf;
  const size_t chunk = (size_t)256 << 20;
  for (size_t off = 0; ok && off < total; off += chunk) {
    const size_t nb = std::min(chunk, total - off);
    buf.resize(nb);
    if (hipMemcpy(buf.data(), (uint8_t*)ix->data + off, nb, hipMemcpyDeviceToHost) != hipSuccess) {
      fclose(f);
      return fail(RFX_EDEVICE, "hipMemcpy D2H failed while saving");
    }
    ok = fwrite(buf.data(), 1, nb, f) == nb;
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok) return fail(RFX_EIO, "write failed for %s", tmp.c_str());
  if (rename(tmp.c_str(), path) != 0) return fail(RFX_EIO, "rename to %s failed", path);
  return RFX_OK;
}

int rfx_index_load(const char* path, int device, rfx_index_t* out) {
  if (!path || !out) return fail(RFX_EINVAL, "null path / out");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(RFX_EIO, "cannot open %s", path);
  char magic[8];
  uint32_t hdr[4];
  int64_t cnt[2];
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "RFXIDX01", 8) != 0 || fread(hdr, 4, 4, f) != 4 ||
      fread(cnt, 8, 2, f) != 2 || hdr[0] != 1u) {
    fclose(f);
    return fail(RFX_EIO, "%s is not an rfx index file", path);
  }
  rfx_index_t h = 0;
  int rc = rfx_index_create(device, (int)hdr[1], (int)hdr[2], cnt[0], &h);
  if (rc) {
    fclose(f);
    return rc;
  }
  auto ix = get(h);
  const size_t tb = (size_t)(cnt[0] + 7) / 8;
  ix->tomb.assign(tb, 0);
  if (tb && fread(ix->tomb.data(), 1, tb, f) != tb) {
    fclose(f);
    rfx_index_destroy(h);
    return fail(RFX_EIO, "truncated tombstones in %s", path);
  }
  const size_t total = (size_t)cnt[0] * ix->row_bytes();
  std::vector<uint8_t> buf;
  const size_t chunk = (size_t)256 << 20;
  for (size_t off = 0; off < total; off += chunk) {
    const size_t nb = std::min(chunk, total - off);
    buf.resize(nb);
    if (fread(buf.data(), 1, nb, f) != nb) {
      fclose(f);
      rfx_index_destroy(h);
      return fail(RFX_EIO, "truncated rows in %s", path);
    }
    if (hipMemcpy((uint8_t*)ix->data + off, buf.data(), nb, hipMemcpyHostToDevice) != hipSuccess) {
      fclose(f);
      rfx_index_destroy(h);
      return fail(RFX_EDEVICE, "hipMemcpy H2D failed while loading");
    }
  }
  fclose(f);
  ix->rows = cnt[0];
  ix->live = cnt[1];
  *out = h;
  return RFX_OK;
}


// ---- append-only row files (rfx/store.py) --------------------------------------------------------
int rfx_rows_append(rfx_index_t h, const char* path, int64_t row0, int64_t file_base) {
  auto ix = get(h);
  if (!ix || !path) return fail(RFX_EINVAL, "unknown index handle / null path");
  RFX_RLOCK(ix);
  if (row0 < 0 || row0 > ix->rows) return fail(RFX_EINVAL, "row0 %lld outside [0, %lld]", (long long)row0, (long long)ix->rows);
  if (file_base < 0) return fail(RFX_EINVAL, "file_base < 0");
  RFX_HIP(hipSetDevice(ix->device));
  Fd f;
  f.fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  if (f.fd < 0) return fail(RFX_EIO, "cannot open %s: %s", path, strerror(errno));
  uint8_t hdr[kRowsHdr], want[kRowsHdr];
  rows_header(*ix, want);
  struct stat sb;
  if (fstat(f.fd, &sb) != 0) return fail(RFX_EIO, "stat %s: %s", path, strerror(errno));
  if (sb.st_size >= kRowsHdr) {
    if (!full_pread(f.fd, hdr, kRowsHdr, 0) || memcmp(hdr, want, kRowsHdr) != 0)
      return fail(RFX_EIO, "%s is not a row file of this index's dim/dtype", path);
  } else if (file_base + row0 != 0) {
    return fail(RFX_EIO, "%s holds no rows, cannot append at row %lld", path, (long long)(file_base + row0));
  } else if (pwrite(f.fd, want, kRowsHdr, 0) != kRowsHdr) {
    return fail(RFX_EIO, "header write to %s failed", path);
  } else {
    sb.st_size = kRowsHdr;
  }
  const int64_t rb = ix->row_bytes();
  const off_t at = kRowsHdr + (file_base + row0) * rb;
  if (sb.st_size < at) return fail(RFX_EIO, "%s holds fewer than %lld rows", path, (long long)(file_base + row0));
  if (ftruncate(f.fd, at) != 0) return fail(RFX_EIO, "truncate %s: %s", path, strerror(errno));
  if (lseek(f.fd, at, SEEK_SET) < 0) return fail(RFX_EIO, "seek %s failed", path);
  const size_t total = (size_t)(ix->rows - row0) * rb;
  if (total) {
    Pinned buf(std::min(total, kStage));
    if (!buf.p) return fail(RFX_ENOMEM, "pinned staging buffer");
    for (size_t off = 0; off < total; off += kStage) {
      const size_t nb = std::min(kStage, total - off);
      RFX_HIP(hipMemcpy(buf.p, (uint8_t*)ix->data + row0 * rb + off, nb, hipMemcpyDeviceToHost));
      if (!full_write(f.fd, (const uint8_t*)buf.p, nb)) return fail(RFX_EIO, "write to %s failed", path);
    }
  }
  if (fsync(f.fd) != 0) return fail(RFX_EIO, "fsync %s: %s", path, strerror(errno));
  return RFX_OK;
}

int rfx_rows_sync(rfx_index_t h, const char* path, int64_t upto, int64_t file_base) {
  auto ix = get(h);
  if (!ix || !path) return fail(RFX_EINVAL, "unknown index handle / null path");
  RFX_WLOCK(ix);
  if (upto < ix->rows) return fail(RFX_EINVAL, "upto %lld < rows %lld", (long long)upto, (long long)ix->rows);
  if (upto == ix->rows) return RFX_OK;
  if (file_base < 0) return fail(RFX_EINVAL, "file_base < 0");
  RFX_HIP(hipSetDevice(ix->device));
  Fd f;
  f.fd = open(path, O_RDONLY | O_CLOEXEC);
  if (f.fd < 0) return fail(RFX_EIO, "cannot open %s: %s", path, strerror(errno));
  uint8_t hdr[kRowsHdr], want[kRowsHdr];
  rows_header(*ix, want);
  if (!full_pread(f.fd, hdr, kRowsHdr, 0) || memcmp(hdr, want, kRowsHdr) != 0)
    return fail(RFX_EIO, "%s is not a row file of this index's dim/dtype", path);
  const int64_t rb = ix->row_bytes();
  struct stat sb;
  if (fstat(f.fd, &sb) != 0 || sb.st_size < kRowsHdr + (file_base + upto) * rb)
    return fail(RFX_EIO, "%s holds fewer than %lld rows", path, (long long)(file_base + upto));
  int rc = grow(*ix, upto, nullptr);
  if (rc) return rc;
  // two pinned buffers: read the next block from the file while the previous one is copied up
  const size_t total = (size_t)(upto - ix->rows) * rb;
  Pinned b0(std::min(total, kStage)), b1(std::min(total, kStage));
  if (!b0.p || !b1.p) return fail(RFX_ENOMEM, "pinned staging buffers");
  hipStream_t st;
  RFX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev[2];
  RFX_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  RFX_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  void* bufs[2] = {b0.p, b1.p};
  bool used[2] = {false, false};
  const off_t src0 = kRowsHdr + (file_base + ix->rows) * rb;
  uint8_t* dst0 = (uint8_t*)ix->data + ix->rows * rb;
  int err = RFX_OK;
  for (size_t off = 0, i = 0; off < total && err == RFX_OK; off += kStage, i ^= 1) {
    const size_t nb = std::min(kStage, total - off);
    if (used[i] && hipEventSynchronize(ev[i]) != hipSuccess) err = fail(RFX_EDEVICE, "staging event");
    if (err == RFX_OK && !full_pread(f.fd, (uint8_t*)bufs[i], nb, src0 + (off_t)off))
      err = fail(RFX_EIO, "read from %s failed", path);
    if (err == RFX_OK && (hipMemcpyAsync(dst0 + off, bufs[i], nb, hipMemcpyHostToDevice, st) != hipSuccess ||
                          hipEventRecord(ev[i], st) != hipSuccess))
      err = fail(RFX_EDEVICE, "H2D copy failed");
    used[i] = true;
  }
  if (hipStreamSynchronize(st) != hipSuccess && err == RFX_OK) err = fail(RFX_EDEVICE, "H2D copy failed");
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  (void)hipStreamDestroy(st);
  if (err) {
    // rows beyond ix->rows may be partly written: restore the NaN tail invariant
    fill_tail_nan(*ix, nullptr);
    return err;
  }
  const int64_t n = upto - ix->rows, first = ix->rows;
  ix->rows = upto;
  ix->live += n;
  ix->tomb.resize((size_t)(ix->rows + 7) / 8, 0);
  return screen_update(*ix, first, nullptr);
}

// ---- search ---------------------------------------------------------------------------------------
int rfx_search_workspace_bytes(rfx_index_t h, int64_t nq, int k, size_t* out_bytes) {
  auto ix = get(h);
  if (!ix || !out_bytes) return fail(RFX_EINVAL, "unknown index handle / null out");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);  // >= every scan layout's workspace too
  if (rc) return rc;
  *out_bytes = L.total;
  return RFX_OK;
}

int rfx_scan_plan(rfx_index_t h, int64_t nq, int k, int* out_kernel, int64_t* out_n_cand) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (out_kernel) *out_kernel = L.kernel;
  if (out_n_cand) *out_n_cand = L.n_cand;
  return RFX_OK;
}

int rfx_scan_topk(rfx_index_t h, const void* queries_d, int64_t nq, int k, float* cand_scores_d,
                  int32_t* cand_rows_d, void* ws_d, size_t ws_bytes, void* stream) {
  return rfx_scan_topk_masked(h, queries_d, nq, k, nullptr, 0, cand_scores_d, cand_rows_d, ws_d, ws_bytes, stream);
}

int rfx_scan_topk_masked(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                         int64_t mask_words, float* cand_scores_d, int32_t* cand_rows_d, void* ws_d, size_t ws_bytes,
                         void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (ws_bytes < scan_ws_bytes(L) || !ws_d) return fail(RFX_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, scan_ws_bytes(L));
  if (nq > 0 && !queries_d) return fail(RFX_EINVAL, "null queries");
  if (row_mask_d && mask_words < (ix->rows + 31) / 32)
    return fail(RFX_EINVAL, "row mask has %lld words, the index needs %lld", (long long)mask_words,
                (long long)((ix->rows + 31) / 32));
  RFX_HIP(hipSetDevice(ix->device));
  return scan_into(*ix, L, queries_d, nq, cand_scores_d, cand_rows_d, (uint8_t*)ws_d, (hipStream_t)stream, row_mask_d);
}

int rfx_topk_merge(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64, int64_t nq, int64_t n_cand,
                   int k, int64_t row_offset, float* out_scores_d, int64_t* out_rows_d, void* stream) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0 || n_cand < 0) return fail(RFX_EINVAL, "negative sizes");
  if (nq > 0 && (!out_scores_d || !out_rows_d)) return fail(RFX_EINVAL, "null outputs");
  if (rfx::launch_topk_merge(cand_scores_d, cand_rows_d, rows_are_i64, nq, n_cand, k, row_offset, out_scores_d,
                             out_rows_d, (hipStream_t)stream) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_scan_list_len(rfx_index_t h, int64_t nq, int k, int* out_list_len) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (!out_list_len) return fail(RFX_EINVAL, "null out");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_layout(*ix, nq, k, L);
  if (rc) return rc;
  *out_list_len = L.kernel ? L.mp.k_lane : L.vp.k_slot;
  return RFX_OK;
}

int rfx_topk_merge_lists(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64, int64_t nq,
                         int64_t n_cand, int list_len, int k, int64_t row_offset, float* out_scores_d,
                         int64_t* out_rows_d, void* stream) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0 || n_cand < 0 || list_len < 1) return fail(RFX_EINVAL, "negative sizes / list_len < 1");
  if (n_cand >= INT32_MAX) return fail(RFX_EINVAL, "n_cand must be < 2^31");
  if (nq > 0 && (!out_scores_d || !out_rows_d)) return fail(RFX_EINVAL, "null outputs");
  if (rfx::launch_topk_merge_lists(cand_scores_d, cand_rows_d, rows_are_i64, nq, n_cand, list_len, k, row_offset,
                                   out_scores_d, out_rows_d, nullptr, (hipStream_t)stream) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_rescore_topk(rfx_index_t h, const void* queries_d, int64_t nq, int k, int64_t row_offset, float* scores_d,
                     int64_t* rows_d, void* records_d, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0) return fail(RFX_EINVAL, "nq < 0");
  if (nq > 0 && (!queries_d || (!records_d && (!scores_d || !rows_d))))
    return fail(RFX_EINVAL, "null queries / answer");
  RFX_RLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  const rfx::Rescore rs{ix->data, queries_d, ix->dim, ix->dtype, ix->rows};
  rfx::launch_rescore_topk(rs, nq, k, row_offset, records_d ? nullptr : scores_d, records_d ? nullptr : rows_d,
                           records_d, (hipStream_t)stream);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_topk_merge_records(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64, int64_t nq,
                           int64_t n_cand, int list_len, int k, int64_t row_offset, void* out_records_d,
                           void* stream) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0 || n_cand < 0 || list_len < 1) return fail(RFX_EINVAL, "negative sizes / list_len < 1");
  if (n_cand >= INT32_MAX) return fail(RFX_EINVAL, "n_cand must be < 2^31");
  if (nq > 0 && !out_records_d) return fail(RFX_EINVAL, "null output");
  if (rfx::launch_topk_merge_lists(cand_scores_d, cand_rows_d, rows_are_i64, nq, n_cand, list_len, k, row_offset,
                                   nullptr, nullptr, out_records_d, (hipStream_t)stream) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_topk_merge_sorted(const float* cand_scores_d, const void* cand_rows_d, int rows_are_i64, int64_t nq,
                          int64_t n_cand, int list_len, int k, int64_t row_offset, float* out_scores_d,
                          int64_t* out_rows_d, void* out_records_d, void* stream) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nq < 0 || n_cand < 0 || list_len < 1) return fail(RFX_EINVAL, "negative sizes / list_len < 1");
  if (n_cand >= INT32_MAX) return fail(RFX_EINVAL, "n_cand must be < 2^31");
  if (n_cand % list_len) return fail(RFX_EINVAL, "n_cand %% list_len != 0");
  if (nq > 0 && !out_records_d && (!out_scores_d || !out_rows_d)) return fail(RFX_EINVAL, "null outputs");
  if (rfx::launch_topk_merge_lists(cand_scores_d, cand_rows_d, rows_are_i64, nq, n_cand, list_len, k, row_offset,
                                   out_records_d ? nullptr : out_scores_d, out_records_d ? nullptr : out_rows_d,
                                   out_records_d, (hipStream_t)stream, /*sorted=*/true) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_merge_gathered(const void* records_d, int world, int64_t nq, int k, float* out_scores_d, int64_t* out_rows_d,
                       void* stream) {
  if (k < 1 || k > 64) return fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (world < 1 || nq < 0) return fail(RFX_EINVAL, "world < 1 or nq < 0");
  if (nq > 0 && (!records_d || !out_scores_d || !out_rows_d)) return fail(RFX_EINVAL, "null buffers");
  if (rfx::launch_merge_gathered(records_d, world, nq, k, out_scores_d, out_rows_d, (hipStream_t)stream) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

#ifdef RFX_DEBUG_BUILD
// ---- debug build only (librfx_dbg.so, `make dbg`; tools/) ------------------------------------
// Diagnostic entry point (not in include/rfx.h): the bf16 / nq 256 / k 10 MFMA scan with
// parts of the kernel removed, for profiling (mode 1 = no top-k epilogue, 2 = no MFMA).
int rfx_dbg_scan_variant(rfx_index_t h, const void* queries_d, int64_t nq, int k, int mode, float* cs, int32_t* cr,
                         void* ws_d, size_t ws_bytes, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (L.kernel == 0 || ws_bytes < scan_ws_bytes(L)) return fail(RFX_EINVAL, "variant needs an MFMA plan");
  hipStream_t st = (hipStream_t)stream;
  void* qpad = (uint8_t*)ws_d + L.q_off;
  rfx::launch_pad_queries(queries_d, nq, L.mp.nq_pad, ix->dim, 2, qpad, st);
  int rc2;
  if (mode >= 20000000)  // headline kernel (k_scan_mfma6.h) ablations: mode 20000000 + MODE
    rc2 = rfx::launch_scan_mfma6_dbg(rfx::plan_scan_mfma6(ix->rows, ix->dim, ix->dtype, nq, k), mode - 20000000, ix->data,
                                     (int)ix->rows, ix->dtype, qpad, (int)nq, (uint32_t*)((uint8_t*)ws_d + L.tau_off), cs, cr, st);
  else if (mode >= 10 && mode < 20)  // 256x256 kernel ablations: mode 10 + MODE
    rc2 = rfx::launch_scan_mfma2_dbg(rfx::plan_scan_mfma2(ix->rows, ix->dim, ix->dtype, nq, k), mode - 10, ix->data,
                                     (int)ix->rows, ix->dim, qpad, (int)nq, (uint32_t*)((uint8_t*)ws_d + L.tau_off),
                                     cs, cr, st);
  else if (mode == 3)  // the production kernel for this plan
    return scan_into(*ix, L, queries_d, nq, cs, cr, (uint8_t*)ws_d, st);
  else
    rc2 = rfx::launch_scan_mfma_dbg(rfx::plan_scan_mfma(ix->rows, ix->dim, ix->dtype, nq, k), mode, ix->data,
                                    (int)ix->rows, ix->dim, qpad, (int)nq, cs, cr, st);
  if (rc2 != 0) return fail(RFX_EUNSUPPORTED, "variant unsupported for this plan");
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

}  // extern "C"
namespace rfx {
int dbg_select_times(unsigned long long* out_h);
int dbg_k11_times(unsigned long long* blocks_h, unsigned long long* last_h);
int dbg_k10_block_times(unsigned long long* out_h);
int dbg_k10_trips(unsigned int* out_h, int reset);
constexpr int k10_tau_words() { return 16; }  // k_scan_screen.h kTauW
int launch_scan_screen_dbg(const MfmaPlan& p, int variant, const int8_t* X, const void* tmv, const uint32_t* sts,
                           int nrows, const int8_t* Qc, const float* qe2, int nq, uint32_t* tau, float* cs, int* cr,
                           uint32_t* dr, hipStream_t st);
}
extern "C" {
// Diagnostic (k10_dbg.hip): the two-pass scan's query quantiser + one kernel-10 variant
// (100000 * RING + MODE), or variant 9: a plain streaming read of the int8 copy (its HBM ceiling).
int rfx_dbg_screen_variant(rfx_index_t h, const void* queries_d, int64_t nq, int k, int variant, void* ws_d,
                           size_t ws_bytes, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (L.kernel != 10 || ws_bytes < L.total) return fail(RFX_EINVAL, "variant needs a two-pass plan and its workspace");
  hipStream_t st = (hipStream_t)stream;
  uint8_t* ws = (uint8_t*)ws_d;
  if (variant == 9) {
    rfx::launch_stream_read(ix->scodes, ix->rows * ix->dim, (uint32_t*)(ws + L.s_gate), st);
    RFX_HIP(hipGetLastError());
    return RFX_OK;
  }
  int8_t* qc = (int8_t*)(ws + L.s_qc);
  float* qe2 = (float*)(ws + L.s_qe2);
  uint32_t* stau = (uint32_t*)(ws + L.s_tau);
  rfx::ScreenSeed sd;
  sd.X8 = ix->scodes;
  sd.tmeta = ix->smeta;
  sd.nrows = (int)ix->rows;
  sd.kl = L.sp.k_lane;
  rfx::launch_screen_queries(queries_d, ix->dtype, ix->dim, nq, L.sp.nq_pad, qc, qe2, ix->sstats, stau,
                             (uint32_t*)(ws + L.s_gate), nullptr, 0, st, &sd);
  // RFX_DBG_KEEP_TAU=1: the slot table starts from the previous launch's final one (the same queries on
  // the same rows: still a lower bound of a_k) — the timing of a bound with no warm-up at all
  static const bool keep_tau = getenv("RFX_DBG_KEEP_TAU") != nullptr;
  static uint32_t* tau_saved = nullptr;
  static size_t tau_saved_bytes = 0;
  const size_t tb = rfx::tau_bytes_screen(L.sp);
  if (keep_tau) {
    if (tau_saved_bytes < tb) {
      if (tau_saved) RFX_HIP(hipFree(tau_saved));
      RFX_HIP(hipMalloc(&tau_saved, tb));
      RFX_HIP(hipMemsetAsync(tau_saved, 0, tb, st));
      tau_saved_bytes = tb;
    }
    RFX_HIP(hipMemcpyAsync(stau, tau_saved, tb, hipMemcpyDeviceToDevice, st));
  }
  if (rfx::launch_scan_screen_dbg(L.sp, variant, ix->scodes, ix->smeta, ix->sstats, (int)ix->rows, qc, qe2, (int)nq, stau,
                                  (float*)(ws + L.s_cs), (int*)(ws + L.s_cr), (uint32_t*)(ws + L.s_drop), st) != 0)
    return fail(RFX_EUNSUPPORTED, "screen variant %d unsupported", variant);
  RFX_HIP(hipGetLastError());
  if (keep_tau) RFX_HIP(hipMemcpyAsync(tau_saved, stau, tb, hipMemcpyDeviceToDevice, st));
  return RFX_OK;
}

// Diagnostic: the two-pass search with a kernel-10 variant (quantiser, the variant, select; no gated
// fallback: *fallback_h says whether it would have run): the variant's answer against production's.
int rfx_dbg_screen_search(rfx_index_t h, const void* queries_d, int64_t nq, int k, int variant, float* out_s,
                          int64_t* out_r, void* ws_d, size_t ws_bytes, void* stream, uint32_t* fallback_h) {
  auto ix = get(h);
  if (!ix || !fallback_h) return fail(RFX_EINVAL, "unknown index handle / null out");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (L.kernel != 10 || ws_bytes < L.total) return fail(RFX_EINVAL, "variant needs a two-pass plan and its workspace");
  hipStream_t st = (hipStream_t)stream;
  uint8_t* ws = (uint8_t*)ws_d;
  int8_t* qc = (int8_t*)(ws + L.s_qc);
  float* qe2 = (float*)(ws + L.s_qe2);
  uint32_t* stau = (uint32_t*)(ws + L.s_tau);
  uint32_t* gate = (uint32_t*)(ws + L.s_gate);
  rfx::ScreenSeed sd;
  sd.X8 = ix->scodes;
  sd.tmeta = ix->smeta;
  sd.nrows = (int)ix->rows;
  sd.kl = L.sp.k_lane;
  rfx::launch_screen_queries(queries_d, ix->dtype, ix->dim, nq, L.sp.nq_pad, qc, qe2, ix->sstats, stau, gate, nullptr, 0,
                             st, &sd);
  if (rfx::launch_scan_screen_dbg(L.sp, variant, ix->scodes, ix->smeta, ix->sstats, (int)ix->rows, qc, qe2, (int)nq, stau,
                                  (float*)(ws + L.s_cs), (int*)(ws + L.s_cr), (uint32_t*)(ws + L.s_drop), st) != 0)
    return fail(RFX_EUNSUPPORTED, "screen variant %d unsupported", variant);
  const void* qpad = queries_d;
  if (nq != L.mp.nq_pad || ((uintptr_t)queries_d & 15)) {
    qpad = ws + L.q_off;
    rfx::launch_pad_queries(queries_d, nq, L.mp.nq_pad, ix->dim, 2, (void*)qpad, st);
  }
  if (rfx::launch_screen_select((float*)(ws + L.s_cs), (int*)(ws + L.s_cr), (uint32_t*)(ws + L.s_drop), L.sp.n_lists,
                                L.sp.k_lane, qe2, qpad, ix->data, ix->dim, ix->dtype, nq, k, 0, out_s, out_r, nullptr, gate,
                                (int*)(ws + L.s_diag), 0, st) != 0)
    return fail(RFX_EUNSUPPORTED, "screen select k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  RFX_HIP(hipStreamSynchronize(st));
  RFX_HIP(hipMemcpy(fallback_h, gate, 4, hipMemcpyDeviceToHost));
  return RFX_OK;
}

// Diagnostic: after a kernel-10 variant with MODE 32, the slow-path entries it counted (sum over waves).
int rfx_dbg_screen_counts(rfx_index_t h, int64_t nq, int k, const void* ws_d, uint64_t* out) {
  auto ix = get(h);
  if (!ix || !out) return fail(RFX_EINVAL, "unknown index handle / null out");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (L.kernel != 10) return fail(RFX_EINVAL, "not a two-pass plan");
  std::vector<uint32_t> t((size_t)L.sp.nq_pad * rfx::k10_tau_words());
  RFX_HIP(hipMemcpy(t.data(), (const uint8_t*)ws_d + L.s_tau, t.size() * 4, hipMemcpyDeviceToHost));
  uint64_t n = 0;
  for (size_t q = 0; q < (size_t)L.sp.nq_pad; ++q) n += t[q * rfx::k10_tau_words() + 15];
  *out = n;
  return RFX_OK;
}

// Diagnostic: the select kernel's per-block phase clocks of its last launch (k_screen.hip g_sel_t:
// [256][8] u64, 100-MHz wall clock; phases 0 start, 1 candidates compacted, 2 a_k, 3 survivors,
// 4 re-scored, 5 written).
int rfx_dbg_select_times(unsigned long long* out_h) {
  if (!out_h) return fail(RFX_EINVAL, "null out");
  if (rfx::dbg_select_times(out_h) != 0) return fail(RFX_EDEVICE, "hipMemcpyFromSymbol failed");
  return RFX_OK;
}

// Diagnostic: kernel 10's per-block wall clocks of the last MODE-65536 variant launch (k10_dbg.hip
// g_k10_bt: [1024][4] u64: wall clock start / end (100 MHz), shader clock start / end).
int rfx_dbg_k10_block_times(unsigned long long* out_h) {
  if (!out_h) return fail(RFX_EINVAL, "null out");
  if (rfx::dbg_k10_block_times(out_h) != 0) return fail(RFX_EDEVICE, "hipMemcpyFromSymbol failed");
  return RFX_OK;
}

// Diagnostic: kernel 10's slow-path entries and trips per tile index (debug MODE 8192, k10_dbg.hip
// g_k10_trips [2][64], summed over launches since the last reset; reset != 0 zeroes them).
int rfx_dbg_k10_trips(unsigned int* out_h, int reset) {
  if (!out_h && !reset) return fail(RFX_EINVAL, "null out");
  if (rfx::dbg_k10_trips(out_h, reset) != 0) return fail(RFX_EDEVICE, "hipMemcpy(From|To)Symbol failed");
  return RFX_OK;
}

// Diagnostic: kernel 11's phase clocks of its last launch (k_screen_valu.hip g_k11_t [1024][4] per
// block, g_k11_last [8] for the last block; 100-MHz wall clock).
int rfx_dbg_k11_times(unsigned long long* blocks_h, unsigned long long* last_h) {
  if (!blocks_h || !last_h) return fail(RFX_EINVAL, "null out");
  if (rfx::dbg_k11_times(blocks_h, last_h) != 0) return fail(RFX_EDEVICE, "hipMemcpyFromSymbol failed");
  return RFX_OK;
}

// Diagnostic: read the whole index once with a plain dwordx4 streaming kernel (HBM ceiling).
int rfx_dbg_stream_read(rfx_index_t h, void* scratch4_d, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  rfx::launch_stream_read(ix->data, ix->rows * ix->row_bytes(), (uint32_t*)scratch4_d, (hipStream_t)stream);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

#endif  // RFX_DEBUG_BUILD

int rfx_search(rfx_index_t h, const void* queries_d, int64_t nq, int k, float* out_scores_d, int64_t* out_rows_d,
               void* ws_d, size_t ws_bytes, void* stream) {
  return rfx_search_masked(h, queries_d, nq, k, nullptr, 0, out_scores_d, out_rows_d, ws_d, ws_bytes, stream);
}

}  // extern "C"

namespace {
// One search (every rfx_search* entry point): writes (out_s, out_r) or, with out_rec, merge
// records with row_offset added.  ev0 / ev1 (hipEvent_t, optional) are recorded on the stream
// right before and after the scan kernel (the two-pass scan's int8 screen; the exact scan; the
// one-launch VALU search as a whole): the benchmark's per-kernel timing.
int search_impl(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d, int64_t mask_words,
                int64_t row_offset, float* out_scores_d, int64_t* out_rows_d, void* out_rec, void* ws_d, size_t ws_bytes,
                void* stream, void* ev0, void* ev1, int stages = 3, int scan_blocks = 0) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (stages < 1 || stages > 3) return fail(RFX_EINVAL, "stages %d: bit 1 scan, bit 2 select", stages);
  if (scan_blocks < 0 || scan_blocks > 256) return fail(RFX_EINVAL, "scan_blocks %d out of [0, 256]", scan_blocks);
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L, scan_blocks);
  if (rc) return rc;
  if (ws_bytes < L.total || (L.total && !ws_d)) return fail(RFX_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, L.total);
  if (nq > 0 && (!queries_d || (!out_rec && (!out_scores_d || !out_rows_d)))) return fail(RFX_EINVAL, "null queries / outputs");
  if (row_mask_d && mask_words < (ix->rows + 31) / 32)
    return fail(RFX_EINVAL, "row mask has %lld words, the index needs %lld", (long long)mask_words,
                (long long)((ix->rows + 31) / 32));
  RFX_HIP(hipSetDevice(ix->device));
  hipStream_t st = (hipStream_t)stream;
  uint8_t* ws = (uint8_t*)ws_d;
  auto mark = [&](void* ev) -> int {
    if (ev) RFX_HIP(hipEventRecord((hipEvent_t)ev, st));
    return RFX_OK;
  };
  if (L.kernel == 10)
    return screen_search(*ix, L, queries_d, nq, k, row_mask_d, row_offset, out_scores_d, out_rows_d, out_rec, ws, st,
                         ev0, ev1, stages);
  if (!(stages & 1)) return RFX_OK;  // another plan: the whole search is stage 1
  if (nq == 0) return RFX_OK;
  float* cs = (float*)(ws + L.cs_off);
  int32_t* cr = (int32_t*)(ws + L.cr_off);
  // a records / row-offset output (a shard of a sharded store) of the one-launch searches: their
  // (score, row) pairs go to the workspace, then one pack launch writes the caller's output
  const bool pack = out_rec || row_offset != 0;
  float* vo_s = pack ? (float*)(ws + L.pk_off) : out_scores_d;
  int64_t* vo_r = pack ? (int64_t*)(ws + L.pk_r_off) : out_rows_d;
  auto finish_pack = [&]() -> int {
    if (!pack) return RFX_OK;
    rfx::launch_pack_records(vo_s, vo_r, nq * k, row_offset, out_rec, out_scores_d, out_rows_d, st);
    RFX_HIP(hipGetLastError());
    return RFX_OK;
  };
  if ((!pack || L.pk_off) && screen_valu_eligible(*ix, L, nq, k) && ((uintptr_t)queries_d & 15) == 0) {
    uint32_t* state = nullptr;
    std::unique_lock<std::mutex> slk(ix->state_mu);  // held until the launches are enqueued
    if ((rc = fused_state(*ix, st, &state, slk))) return rc;
    uint32_t* sv = state + rfx::kScreenValuState;
    K11Order& ko = k11_order(ix->device);
    std::lock_guard<std::mutex> olk(ko.mu);
    if (!ko.ev) RFX_HIP(hipEventCreateWithFlags(&ko.ev, hipEventDisableTiming));
    if (ko.used && ko.last != st) {
      ko.multi = true;
      ko.same = 0;
      if (ko.recorded && !k11_unordered()) RFX_HIP(hipStreamWaitEvent(st, ko.ev, 0));
    } else if (ko.multi && ++ko.same >= kK11OrderDecay) {
      ko.multi = false;
      ko.recorded = false;
    }
    if ((rc = mark(ev0))) return rc;
    // one launch for a lone question: the screen, and the exact one-launch search run by the same
    // launch when the screen cannot prove its answer (its state: the front of the same search state)
    if (rfx::launch_screen_valu(L.vp, ix->scodes, ix->smeta, ix->sstats, (int)ix->rows, ix->dim, ix->dtype, ix->data,
                                queries_d, (int)nq, row_mask_d, sv, state, cs, cr, (uint32_t*)(ws + L.cx_off), k,
                                vo_s, vo_r,
                                (ix->screen == 2 ? 1 : 0) | k11_ablate(), st) != 0)
      return fail(RFX_EUNSUPPORTED, "two-pass VALU search launch rejected");
    if (ko.multi) {
      RFX_HIP(hipEventRecord(ko.ev, st));
      ko.recorded = true;
    }
    ko.last = st;
    ko.used = true;
    if ((rc = mark(ev1))) return rc;
    if (!rfx::screen_valu_inline_fallback(nq == 1 ? 1 : 8, ix->dtype, ix->dim)) {
      // several questions (or f32 rows at d 1024): the exact one-launch search, gated on the word the
      // screen's last block wrote
      if (rfx::launch_search_valu_fused(L.vp, ix->data, (int)ix->rows, ix->dim, ix->dtype, queries_d, (int)nq, cs, cr,
                                        state, k, vo_s, vo_r, st, row_mask_d, sv + 24) != 0)
        return fail(RFX_EUNSUPPORTED, "VALU search launch rejected");
    }
    RFX_HIP(hipGetLastError());
    slk.unlock();
    return finish_pack();
  }
  // (the one-launch kernel reads the caller's queries with 16-B loads: an unaligned buffer takes
  // the three-launch path, whose widening copy is aligned)
  if ((!pack || L.pk_off) && L.kernel == 0 && ix->rows > 0 && nq <= rfx::kValuFusedMaxNq && fused_enabled() &&
      ((uintptr_t)queries_d & 15) == 0) {
    uint32_t* state = nullptr;
    std::unique_lock<std::mutex> slk(ix->state_mu);  // held until the launch is enqueued
    if ((rc = fused_state(*ix, st, &state, slk))) return rc;
    if ((rc = mark(ev0))) return rc;
    if (rfx::launch_search_valu_fused(L.vp, ix->data, (int)ix->rows, ix->dim, ix->dtype, queries_d, (int)nq, cs, cr,
                                      state, k, vo_s, vo_r, st, row_mask_d) != 0)
      return fail(RFX_EUNSUPPORTED, "VALU search launch rejected");
    RFX_HIP(hipGetLastError());
    slk.unlock();
    if ((rc = mark(ev1))) return rc;
    return finish_pack();
  }
  int64_t n_cand = L.n_cand;
  int list_len = L.kernel ? L.mp.k_lane : L.vp.k_slot;
  if (ix->rows == 0 || n_cand == 0) {  // an empty index: padding only
    n_cand = 0;
    list_len = 1;
  } else {
    if ((rc = mark(ev0))) return rc;
    rc = scan_into(*ix, L, queries_d, nq, cs, cr, ws, st, row_mask_d);
    if (rc) return rc;
    if ((rc = mark(ev1))) return rc;
  }
  // the scan's candidates are sorted lists: the merge bounds admission by the lists' k-th entries; its
  // final top-k is re-scored by the score rule of every plan (fl32 of the f64 dot; k_scan_valu.h)
  const rfx::Rescore rs{ix->data, queries_d, ix->dim, ix->dtype, ix->rows};
  if (rfx::launch_topk_merge_lists(cs, cr, 0, nq, n_cand, list_len, k, row_offset, out_rec ? nullptr : out_scores_d,
                                   out_rec ? nullptr : out_rows_d, out_rec, st, /*sorted=*/n_cand > 0, nullptr,
                                   n_cand > 0 ? &rs : nullptr) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}
}  // namespace

extern "C" {

int rfx_search_masked(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                      int64_t mask_words, float* out_scores_d, int64_t* out_rows_d, void* ws_d, size_t ws_bytes,
                      void* stream) {
  return search_impl(h, queries_d, nq, k, row_mask_d, mask_words, 0, out_scores_d, out_rows_d, nullptr, ws_d, ws_bytes,
                     stream, nullptr, nullptr);
}

int rfx_search_records(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                       int64_t mask_words, int64_t row_offset, void* out_records_d, void* ws_d, size_t ws_bytes,
                       void* stream) {
  if (nq > 0 && !out_records_d) return fail(RFX_EINVAL, "null output");
  return search_impl(h, queries_d, nq, k, row_mask_d, mask_words, row_offset, nullptr, nullptr, out_records_d, ws_d,
                     ws_bytes, stream, nullptr, nullptr);
}

// ---- one search over a row-sharded store, issued from C++ -----------------------------------
}  // extern "C"
namespace {
// The shards' launch sequences are issued by a pool of host threads, one task per shard (one
// thread issuing 8 shards x ~6 launches took ~0.24 ms, ~0.7x of a real 8-GPU step).  The caller's thread
// waits for the ISSUE of every task (not for the GPU), then enqueues the exchange and the merge.  Workers are
// made on first use (at most kIssueThreads) and live for the process; RFX_ISSUE_THREADS=0 keeps the serial
// issue (A/B runs).
constexpr int kIssueThreads = 16;
struct IssuePool {
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::vector<std::thread> workers;
  std::vector<std::function<void()>> tasks;  // this round's tasks; workers take them by index
  size_t next = 0, done = 0;
  uint64_t round = 0;
  std::mutex call_mu;  // one round at a time
  void ensure(size_t n) {
    while (workers.size() < std::min<size_t>(n, kIssueThreads)) {
      workers.emplace_back([this] {
        uint64_t seen = 0;
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return round != seen && next < tasks.size(); });
            f = tasks[next++];
            if (next == tasks.size()) seen = round;
          }
          f();
          std::lock_guard<std::mutex> lk(mu);
          if (++done == tasks.size()) done_cv.notify_all();
        }
      });
      workers.back().detach();
    }
  }
  void run(std::vector<std::function<void()>>& fs) {
    std::lock_guard<std::mutex> call(call_mu);
    ensure(fs.size());
    std::unique_lock<std::mutex> lk(mu);
    tasks.swap(fs);
    next = done = 0;
    ++round;
    cv.notify_all();
    done_cv.wait(lk, [&] { return done == tasks.size(); });
    tasks.clear();
  }
};
IssuePool& issue_pool() {
  static IssuePool* p = new IssuePool();  // (never destroyed: detached workers outlive static destruction)
  return *p;
}
bool parallel_issue() {
  static const bool on = [] {
    const char* e = getenv("RFX_ISSUE_THREADS");
    return !(e && e[0] == '0');
  }();
  return on;
}
// events for the cross-stream orderings of rfx_sharded_search: per thread and device, reused call after
// call (a stream that waited on an event keeps the state it saw when the wait was enqueued)
hipEvent_t pooled_event(int device, int slot) {
  thread_local std::map<int, std::vector<hipEvent_t>> pool;
  auto& v = pool[device];
  while ((int)v.size() <= slot) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    v.push_back(e);
  }
  return v[slot];
}
}  // namespace
extern "C" {

int rfx_sharded_search(int n, const rfx_index_t* handles, const int64_t* bases, const void* queries_d,
                       void* const* qbuf_d, int64_t nq, int k, const uint32_t* const* masks_d,
                       const int64_t* mask_words, void* const* ws_d, const size_t* ws_bytes, void* const* recs_d,
                       void* gathered_d, rfx_comm_t comm, void* src_stream, void* const* streams,
                       float* out_scores_d, int64_t* out_rows_d) {
  if (n < 1 || !handles || !bases || !ws_d || !ws_bytes || !recs_d || !gathered_d || !streams)
    return fail(RFX_EINVAL, "null shard arrays");
  if (k < 1 || k > 64 || nq < 0) return fail(RFX_EINVAL, "k=%d / nq=%lld out of range", k, (long long)nq);
  if (nq == 0) return RFX_OK;
  if (!queries_d || !out_scores_d || !out_rows_d) return fail(RFX_EINVAL, "null queries / outputs");
  std::vector<int> dev(n);
  int64_t qbytes = 0;
  for (int i = 0; i < n; ++i) {
    auto ix = get(handles[i]);
    if (!ix) return fail(RFX_EINVAL, "unknown index handle (shard %d)", i);
    dev[i] = ix->device;
    if (i == 0) qbytes = nq * ix->row_bytes();
    if (!comm && dev[i] != dev[0]) return fail(RFX_EINVAL, "shards on several devices need a communicator");
    // every shard's workspace is checked before anything is enqueued: a regrow-and-retry by the
    // caller then never follows the partial work of the shards before a failing one
    RFX_RLOCK(ix);
    SearchLayout L;
    if (int rc = make_search_layout(*ix, nq, k, L)) return rc;
    if (ws_bytes[i] < L.total || (L.total && !ws_d[i]))
      return fail(RFX_EINVAL, "workspace too small (%zu < %zu, shard %d)", ws_bytes[i], L.total, i);
  }
  const size_t rec_bytes = (size_t)nq * k * 16;
  hipStream_t src = (hipStream_t)src_stream;
  // 1. every shard stream after the queries (one event on the caller's stream)
  int src_dev = dev[0];
  RFX_HIP(hipSetDevice(src_dev));
  hipEvent_t ev = pooled_event(src_dev, 0);
  if (!ev) return fail(RFX_EDEVICE, "hipEventCreate failed");
  RFX_HIP(hipEventRecord(ev, src));
  for (int i = 0; i < n; ++i)
    if ((hipStream_t)streams[i] != src) RFX_HIP(hipStreamWaitEvent((hipStream_t)streams[i], ev, 0));
  // ... and after the previous search's merge on streams[0] (callers reuse the records and gathered buffers
  // from search to search, and the previous merge may still be reading them)
  if (n > 1) {
    RFX_HIP(hipSetDevice(dev[0]));
    hipEvent_t e0 = pooled_event(dev[0], n + 1);
    if (!e0) return fail(RFX_EDEVICE, "hipEventCreate failed");
    RFX_HIP(hipEventRecord(e0, (hipStream_t)streams[0]));
    for (int i = 1; i < n; ++i)
      if ((hipStream_t)streams[i] != (hipStream_t)streams[0]) RFX_HIP(hipStreamWaitEvent((hipStream_t)streams[i], e0, 0));
  }
  // 2. per shard: the queries on its device (a peer copy when it has a buffer there), then its whole search
  // (rfx_search_records: the two-pass scan where the shard holds its int8 copy) into [nq][k] records with its
  // base added — one issue task per shard, run by the pool's threads side by side
  std::vector<int> rcs((size_t)n, RFX_OK);
  std::vector<std::string> errs((size_t)n);
  auto shard_issue = [&](int i) {
    hipStream_t st = (hipStream_t)streams[i];
    int rc = hipSetDevice(dev[i]) == hipSuccess ? RFX_OK : fail(RFX_EDEVICE, "hipSetDevice(%d) failed", dev[i]);
    const void* q = queries_d;
    if (!rc && qbuf_d && qbuf_d[i] && qbuf_d[i] != queries_d) {
      if (hipMemcpyAsync(qbuf_d[i], queries_d, (size_t)qbytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = fail(RFX_EDEVICE, "query copy to shard %d failed", i);
      q = qbuf_d[i];
    }
    if (!rc)
      rc = search_impl(handles[i], q, nq, k, masks_d ? masks_d[i] : nullptr, mask_words ? mask_words[i] : 0, bases[i],
                       nullptr, nullptr, recs_d[i], ws_d[i], ws_bytes[i], st, nullptr, nullptr);
    rcs[i] = rc;
    if (rc) errs[i] = g_err;  // (thread-local: carried back to the caller's thread)
  };
  if (parallel_issue() && n > 1) {
    std::vector<std::function<void()>> fs;
    for (int i = 0; i < n; ++i) fs.push_back([&shard_issue, i] { shard_issue(i); });
    issue_pool().run(fs);
  } else {
    for (int i = 0; i < n; ++i) shard_issue(i);
  }
  for (int i = 0; i < n; ++i)
    if (rcs[i]) return fail(rcs[i], "shard %d: %s", i, errs[i].c_str());
  // 3. the exchange: one RCCL gather to shard 0's device over distinct devices; shards sharing one device
  // stack their records there (in place when recs_d[i] already is row i of gathered_d), ordered by events
  if (comm) {
    std::vector<void*> recvs((size_t)n, nullptr);
    recvs[0] = gathered_d;
    const int rc = rfx_gather_records(comm, (const void* const*)recs_d, recvs.data(), 0, nq, k, streams);
    if (rc) return rc;
  } else {
    RFX_HIP(hipSetDevice(dev[0]));
    for (int i = 0; i < n; ++i) {
      hipStream_t st = (hipStream_t)streams[i];
      uint8_t* dst = (uint8_t*)gathered_d + (size_t)i * rec_bytes;
      if (recs_d[i] != dst) RFX_HIP(hipMemcpyAsync(dst, recs_d[i], rec_bytes, hipMemcpyDeviceToDevice, st));
      if (i > 0 && st != (hipStream_t)streams[0]) {
        hipEvent_t e = pooled_event(dev[0], i);
        if (!e) return fail(RFX_EDEVICE, "hipEventCreate failed");
        RFX_HIP(hipEventRecord(e, st));
        RFX_HIP(hipStreamWaitEvent((hipStream_t)streams[0], e, 0));
      }
    }
  }
  // 4. the gathered merge on shard 0's stream; the caller's stream after it
  RFX_HIP(hipSetDevice(dev[0]));
  if (rfx::launch_merge_gathered(gathered_d, n, nq, k, out_scores_d, out_rows_d, (hipStream_t)streams[0]) != 0)
    return fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  RFX_HIP(hipGetLastError());
  if ((hipStream_t)streams[0] != src) {
    hipEvent_t e = pooled_event(dev[0], n);
    if (!e) return fail(RFX_EDEVICE, "hipEventCreate failed");
    RFX_HIP(hipEventRecord(e, (hipStream_t)streams[0]));
    RFX_HIP(hipStreamWaitEvent(src, e, 0));
  }
  return RFX_OK;
}

int rfx_search_timed(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                     int64_t mask_words, int64_t row_offset, float* out_scores_d, int64_t* out_rows_d,
                     void* out_records_d, void* ws_d, size_t ws_bytes, void* stream, void* ev_scan_begin,
                     void* ev_scan_end) {
  return search_impl(h, queries_d, nq, k, row_mask_d, mask_words, row_offset, out_scores_d, out_rows_d, out_records_d,
                     ws_d, ws_bytes, stream, ev_scan_begin, ev_scan_end);
}

int rfx_search_staged(rfx_index_t h, const void* queries_d, int64_t nq, int k, const uint32_t* row_mask_d,
                      int64_t mask_words, int64_t row_offset, float* out_scores_d, int64_t* out_rows_d,
                      void* out_records_d, void* ws_d, size_t ws_bytes, int stages, int scan_blocks, void* stream) {
  return search_impl(h, queries_d, nq, k, row_mask_d, mask_words, row_offset, out_scores_d, out_rows_d, out_records_d,
                     ws_d, ws_bytes, stream, nullptr, nullptr, stages, scan_blocks);
}

int rfx_stream_create_cu_mask(int device, const uint32_t* cu_mask, int n_words, void** out_stream) {
  if (!cu_mask || n_words < 1 || !out_stream) return fail(RFX_EINVAL, "null mask / out or n_words < 1");
  RFX_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  RFX_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words * 32u, cu_mask));
  *out_stream = (void*)s;
  return RFX_OK;
}

int rfx_stream_destroy(void* stream) {
  if (!stream) return RFX_OK;
  RFX_HIP(hipStreamDestroy((hipStream_t)stream));
  return RFX_OK;
}

int rfx_search_plan(rfx_index_t h, int64_t nq, int k, int* out_kernel) {
  auto ix = get(h);
  if (!ix || !out_kernel) return fail(RFX_EINVAL, "unknown index handle / null out");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);
  if (rc) return rc;
  *out_kernel = screen_valu_eligible(*ix, L, nq, k) ? 11 : L.kernel;
  return RFX_OK;
}

// ---- the int8 screen copy (exact two-pass scan) ------------------------------------------------------
int rfx_index_screen(rfx_index_t h, int mode, void* stream) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  if (mode < 0 || mode > 2) return fail(RFX_EINVAL, "screen mode %d (0 off, 1 on, 2 on + forced fallback)", mode);
  if (mode && !rfx::screen_supported(ix->dim, ix->dtype))
    return fail(RFX_EUNSUPPORTED, "the two-pass scan needs an index of dim 768 or 1024 (dim=%d dtype=%d)",
                ix->dim, ix->dtype);
  hipStream_t st = (hipStream_t)stream;
  RFX_WLOCK(ix);
  RFX_HIP(hipSetDevice(ix->device));
  if (!mode) {
    RFX_HIP(hipDeviceSynchronize());  // no search still reads the copy
    screen_free(*ix);
    ix->screen = 0;
    return RFX_OK;
  }
  const bool had = ix->screen != 0;
  ix->screen = mode;
  if (had && ix->scap == ix->capacity) return RFX_OK;
  const int rc = screen_build(*ix, st);
  if (rc) {
    ix->screen = 0;
    screen_free(*ix);
  } else {
    ix->screen_dropped = 0;
  }
  return rc;
}

int rfx_index_screen_state(rfx_index_t h, int* out_mode, int64_t* out_bytes, int* out_dropped) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  if (out_mode) *out_mode = ix->screen;
  if (out_bytes) *out_bytes = ix->scodes ? screen_bytes(ix->scap, ix->dim) : 0;
  if (out_dropped) *out_dropped = ix->screen_dropped;
  return RFX_OK;
}

int rfx_index_screen_read(rfx_index_t h, int64_t tile0, int64_t ntiles, int8_t* codes_h, float* scales_h,
                          uint32_t* live_h, float* stats_h) {
  auto ix = get(h);
  if (!ix) return fail(RFX_EINVAL, "unknown index handle");
  RFX_RLOCK(ix);
  if (!ix->screen) return fail(RFX_EINVAL, "the index holds no int8 screen copy");
  if (tile0 < 0 || ntiles < 0 || (tile0 + ntiles) * 32 > ix->scap) return fail(RFX_EINVAL, "tiles out of range");
  RFX_HIP(hipSetDevice(ix->device));
  if (codes_h && ntiles)
    RFX_HIP(hipMemcpy(codes_h, ix->scodes + tile0 * 32 * ix->dim, (size_t)ntiles * 32 * ix->dim, hipMemcpyDeviceToHost));
  if ((scales_h || live_h) && ntiles) {
    std::vector<uint32_t> m((size_t)ntiles * 4);
    RFX_HIP(hipMemcpy(m.data(), (const uint8_t*)ix->smeta + tile0 * 16, m.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < ntiles; ++i) {
      if (scales_h) memcpy(scales_h + i, &m[4 * i], 4);
      if (live_h) live_h[i] = m[4 * i + 1];
    }
  }
  if (stats_h) RFX_HIP(hipMemcpy(stats_h, ix->sstats, 12, hipMemcpyDeviceToHost));
  return RFX_OK;
}

int rfx_screen_diag(rfx_index_t h, int64_t nq, int k, const void* ws_d, int32_t* diag_h, uint32_t* fallback_h) {
  auto ix = get(h);
  if (!ix || !ws_d) return fail(RFX_EINVAL, "unknown index handle / null workspace");
  RFX_RLOCK(ix);
  SearchLayout L;
  int rc = make_search_layout(*ix, nq, k, L);
  if (rc) return rc;
  if (L.kernel != 10) return fail(RFX_EINVAL, "the search plan for nq=%lld k=%d is not the two-pass scan", (long long)nq, k);
  RFX_HIP(hipSetDevice(ix->device));
  if (diag_h && nq) RFX_HIP(hipMemcpy(diag_h, (const uint8_t*)ws_d + L.s_diag, (size_t)nq * 8, hipMemcpyDeviceToHost));
  if (fallback_h) RFX_HIP(hipMemcpy(fallback_h, (const uint8_t*)ws_d + L.s_gate, 4, hipMemcpyDeviceToHost));
  return RFX_OK;
}

// ---- embedding -------------------------------------------------------------------------------------
int rfx_embed_weights(int V, int dim, uint64_t seed, void* wt_d, void* stream) {
  if (V <= 0 || (V & (V - 1)) || V % 16 != 0) return fail(RFX_EINVAL, "V=%d must be a power of two >= 16", V);
  if (dim <= 0 || dim % 32 != 0 || dim > 1024) return fail(RFX_EINVAL, "dim=%d must be a multiple of 32 <= 1024", dim);
  if (!wt_d) return fail(RFX_EINVAL, "null weights");
  rfx::launch_embed_weights(V, dim, seed, wt_d, (hipStream_t)stream);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_embed_workspace_bytes(int64_t n, int V, size_t* out_bytes) {
  if (!out_bytes || n < 0 || V <= 0) return fail(RFX_EINVAL, "bad arguments");
  *out_bytes = align_up((size_t)n * V * 2);
  return RFX_OK;
}

int rfx_embed(const int32_t* indptr_d, const int32_t* bucket_d, const int16_t* count_d, int64_t n, int V,
              const void* wt_d, int dim, void* out_d, int out_dtype, void* ws_d, size_t ws_bytes, void* stream) {
  if (n < 0) return fail(RFX_EINVAL, "n < 0");
  if (V <= 0 || (V & (V - 1)) || V % 16 != 0) return fail(RFX_EINVAL, "V=%d must be a power of two >= 16", V);
  if (dim <= 0 || dim % 32 != 0 || dim > 1024) return fail(RFX_EINVAL, "dim=%d must be a multiple of 32 <= 1024", dim);
  if (!valid_dtype(out_dtype)) return fail(RFX_EINVAL, "bad dtype %d", out_dtype);
  if (n == 0) return RFX_OK;
  if (!indptr_d || !bucket_d || !count_d || !wt_d || !out_d) return fail(RFX_EINVAL, "null pointer argument");
  if (ws_bytes < (size_t)n * V * 2) return fail(RFX_EINVAL, "embed workspace too small");
  int rc = rfx::launch_embed(indptr_d, bucket_d, count_d, n, V, wt_d, dim, out_d, out_dtype, ws_d, (hipStream_t)stream);
  if (rc == -2) return fail(RFX_EDEVICE, "hipMemsetAsync failed");
  if (rc) return fail(RFX_EUNSUPPORTED, "embed dim=%d unsupported", dim);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_synth_rows(uint64_t seed, int64_t row0, int64_t n, int dim, int dtype, void* out_d, void* stream) {
  if (n < 0 || row0 < 0 || dim <= 0 || !valid_dtype(dtype)) return fail(RFX_EINVAL, "bad arguments");
  if (n == 0) return RFX_OK;
  if (!out_d) return fail(RFX_EINVAL, "null output");
  rfx::launch_synth_rows(seed, row0, n, dim, dtype, out_d, (hipStream_t)stream);
  RFX_HIP(hipGetLastError());
  return RFX_OK;
}

}  // extern "C"
