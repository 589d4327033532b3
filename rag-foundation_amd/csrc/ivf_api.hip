// ivf_api.hip — C ABI of the IVF-Flat int8 index (include/rfx.h, "IVF-Flat int8").
//
// One handle owns, on one device: the int8 centroid table and its factors, the rows in insertion
// order (int8 codes, dequantisation scale, list label) and — rebuilt lazily after adds — the
// posting lists (codes, scales and row ids in (list, row) order + list offsets).  Kernels:
// k_ivf.hip; numerics: oracle/ivf.py (bit-exact).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "rfx_kernels.h"

namespace {

using rfx::api_fail;

#define IVF_HIP(call)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) return api_fail(RFX_EDEVICE, "%s: %s", #call, hipGetErrorString(e_));   \
  } while (0)

struct Ivf {
  int device = 0, dim = 0, nlist = 0;
  std::mutex mu;
  int8_t* qc = nullptr;  // [nlist][dim]
  float* fc = nullptr;   // [nlist]
  bool trained = false;
  int64_t rows = 0, cap = 0;
  int8_t* codes = nullptr;  // [cap][dim], insertion order
  float* inv = nullptr;     // [cap]
  int* labels = nullptr;    // [cap]
  bool dirty = true;        // posting lists stale
  int64_t lcap = 0;
  int8_t* lcodes = nullptr;  // [lcap rounded up to 64][dim], list order, 64-row blocks chunk-major
  float* linv = nullptr;
  int* lids = nullptr;
  int64_t* off = nullptr;  // [nlist + 1]
  ~Ivf() {
    for (void* p : {(void*)qc, (void*)fc, (void*)codes, (void*)inv, (void*)labels, (void*)lcodes, (void*)linv,
                    (void*)lids, (void*)off})
      if (p) (void)hipFree(p);
  }
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<Ivf>> g_ivf;
std::atomic<uint64_t> g_next{1};

std::shared_ptr<Ivf> get(rfx_ivf_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_ivf.find(h);
  return it == g_ivf.end() ? nullptr : it->second;
}

bool valid_dtype(int dt) { return dt == RFX_F32 || dt == RFX_BF16 || dt == RFX_F16; }

template <class T>
int realloc_copy(T*& p, int64_t old_n, int64_t new_n, size_t per, hipStream_t st) {
  T* q = nullptr;
  if (hipMalloc(&q, (size_t)new_n * per) != hipSuccess) return api_fail(RFX_ENOMEM, "hipMalloc(%zu) failed", (size_t)new_n * per);
  if (p && old_n > 0) IVF_HIP(hipMemcpyAsync(q, p, (size_t)old_n * per, hipMemcpyDeviceToDevice, st));
  IVF_HIP(hipStreamSynchronize(st));
  if (p) IVF_HIP(hipFree(p));
  p = q;
  return RFX_OK;
}

int grow_rows(Ivf& iv, int64_t need, hipStream_t st) {
  if (need <= iv.cap) return RFX_OK;
  int64_t cap = std::max<int64_t>(iv.cap + iv.cap / 2, 4096);
  while (cap < need) cap = cap + cap / 2;
  int rc;
  if ((rc = realloc_copy(iv.codes, iv.rows, cap, (size_t)iv.dim, st))) return rc;
  if ((rc = realloc_copy(iv.inv, iv.rows, cap, sizeof(float), st))) return rc;
  if ((rc = realloc_copy(iv.labels, iv.rows, cap, sizeof(int), st))) return rc;
  iv.cap = cap;
  return RFX_OK;
}

int assign_all(Ivf& iv, int64_t r0, int64_t n, hipStream_t st) {
  if (n <= 0) return RFX_OK;
  if (rfx::ivf::launch_assign(iv.codes + r0 * iv.dim, n, iv.qc, iv.nlist, iv.dim, iv.fc, iv.labels + r0, nullptr, st))
    return api_fail(RFX_EUNSUPPORTED, "assignment launch rejected");
  IVF_HIP(hipGetLastError());
  iv.dirty = true;
  return RFX_OK;
}

int build(Ivf& iv, hipStream_t st) {
  if (!iv.dirty) return RFX_OK;
  const int64_t n = iv.rows;
  if (n > iv.lcap) {
    for (void* p : {(void*)iv.lcodes, (void*)iv.linv, (void*)iv.lids})
      if (p) IVF_HIP(hipFree(p));
    iv.lcodes = nullptr, iv.linv = nullptr, iv.lids = nullptr;
    const int64_t c = std::max<int64_t>(iv.cap, 1);
    // (the list-order codes in whole 64-row blocks: k_ivf.hip gather_rows_kernel)
    if (hipMalloc(&iv.lcodes, (size_t)((c + 63) / 64 * 64) * iv.dim) != hipSuccess ||
        hipMalloc(&iv.linv, (size_t)c * 4) != hipSuccess ||
        hipMalloc(&iv.lids, (size_t)c * 4) != hipSuccess)
      return api_fail(RFX_ENOMEM, "hipMalloc failed for posting lists (%lld rows)", (long long)c);
    iv.lcap = c;
  }
  const size_t tb = rfx::ivf::sort_temp_bytes(std::max<int64_t>(n, 1));
  const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4;
  uint8_t* tmp = nullptr;
  const size_t total = 3 * nb + (size_t)iv.nlist * 4 + tb + 4 * 256;
  if (hipMalloc(&tmp, total) != hipSuccess) return api_fail(RFX_ENOMEM, "hipMalloc(%zu) failed for list build", total);
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  size_t o = 0;
  unsigned* keys_tmp = (unsigned*)(tmp + o);
  o += al(nb);
  int* vals_tmp = (int*)(tmp + o);
  o += al(nb);
  unsigned* keys_out = (unsigned*)(tmp + o);
  o += al(nb);
  int* counts = (int*)(tmp + o);
  o += al((size_t)iv.nlist * 4);
  void* sort_tmp = tmp + o;
  const int rc = rfx::ivf::launch_build_lists(iv.labels, n, iv.nlist, iv.codes, iv.inv, iv.dim, keys_tmp, vals_tmp,
                                              keys_out, iv.lids, sort_tmp, tb, counts, iv.off, iv.lcodes, iv.linv, st);
  const hipError_t e = hipStreamSynchronize(st);
  (void)hipFree(tmp);
  if (rc) return api_fail(RFX_EDEVICE, "posting-list build failed (%d)", rc);
  if (e != hipSuccess) return api_fail(RFX_EDEVICE, "posting-list build: %s", hipGetErrorString(e));
  iv.dirty = false;
  return RFX_OK;
}

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

// list-scan splits per list: enough (list, split) blocks to fill the chip several times over
int ivf_splits(const Ivf& iv) {
  if (const char* e = getenv("RFX_IVF_SPLITS")) {  // tuning override
    const int v = atoi(e);
    if (v >= 1 && v <= 64) return v;
  }
  const int64_t avg = iv.rows / std::max(iv.nlist, 1);
  return avg >= 2048 ? 4 : (avg >= 512 ? 2 : 1);
}

struct IvfLayout {
  int K, splits;
  int64_t ncand;
  size_t qq, qinv, S, Sid, ps, pid, poff, pairs, cs, cr, total;
};

int ivf_layout(const Ivf& iv, int64_t nq, int k, int nprobe, IvfLayout& L) {
  if (k < 1 || k > 64) return api_fail(RFX_EINVAL, "k=%d out of range [1, 64]", k);
  if (nprobe < 1 || nprobe > 64 || nprobe > iv.nlist)
    return api_fail(RFX_EINVAL, "nprobe=%d out of range [1, min(64, nlist=%d)]", nprobe, iv.nlist);
  if (nq < 0 || nq * nprobe > (int64_t)INT32_MAX / 4) return api_fail(RFX_EINVAL, "nq=%lld out of range", (long long)nq);
  L.K = rfx::ivf::list_k(k);
  L.splits = ivf_splits(iv);
  L.ncand = (int64_t)nprobe * L.splits * 4 * L.K;
  size_t o = 0;
  L.qq = o, o += al256((size_t)nq * iv.dim);
  L.qinv = o, o += al256((size_t)nq * 4);
  L.S = o, o += al256((size_t)nq * iv.nlist * 4);
  L.Sid = o, o += al256((size_t)nq * iv.nlist * 4);
  L.ps = o, o += al256((size_t)nq * nprobe * 4);
  L.pid = o, o += al256((size_t)nq * nprobe * 8);
  L.poff = o, o += al256((size_t)(iv.nlist + 1) * 4);
  L.pairs = o, o += al256((size_t)nq * nprobe * 4);
  L.cs = o, o += al256((size_t)nq * L.ncand * 4);
  L.cr = o, o += al256((size_t)nq * L.ncand * 4);
  L.total = o;
  return RFX_OK;
}


// chunked device <-> file copies (persistence)
bool write_dev(FILE* f, const void* d, size_t n) {
  std::vector<uint8_t> buf;
  const size_t chunk = (size_t)256 << 20;
  for (size_t off = 0; off < n; off += chunk) {
    const size_t nb = std::min(chunk, n - off);
    buf.resize(nb);
    if (hipMemcpy(buf.data(), (const uint8_t*)d + off, nb, hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (fwrite(buf.data(), 1, nb, f) != nb) return false;
  }
  return true;
}
bool read_dev(FILE* f, void* d, size_t n) {
  std::vector<uint8_t> buf;
  const size_t chunk = (size_t)256 << 20;
  for (size_t off = 0; off < n; off += chunk) {
    const size_t nb = std::min(chunk, n - off);
    buf.resize(nb);
    if (fread(buf.data(), 1, nb, f) != nb) return false;
    if (hipMemcpy((uint8_t*)d + off, buf.data(), nb, hipMemcpyHostToDevice) != hipSuccess) return false;
  }
  return true;
}

}  // namespace

extern "C" {

int rfx_ivf_create(int device, int dim, int nlist, rfx_ivf_t* out) {
  if (!out) return api_fail(RFX_EINVAL, "null out");
  if (dim < 256 || dim > 1024 || dim % 256) return api_fail(RFX_EINVAL, "IVF dim=%d must be 256, 512, 768 or 1024", dim);
  if (nlist < 1 || nlist > 16384) return api_fail(RFX_EINVAL, "nlist=%d out of range [1, 16384]", nlist);
  IVF_HIP(hipSetDevice(device));
  auto iv = std::make_shared<Ivf>();
  iv->device = device, iv->dim = dim, iv->nlist = nlist;
  if (hipMalloc(&iv->qc, (size_t)nlist * dim) != hipSuccess || hipMalloc(&iv->fc, (size_t)nlist * 4) != hipSuccess ||
      hipMalloc(&iv->off, (size_t)(nlist + 1) * 8) != hipSuccess)
    return api_fail(RFX_ENOMEM, "hipMalloc failed for IVF tables");
  IVF_HIP(hipMemset(iv->off, 0, (size_t)(nlist + 1) * 8));
  const uint64_t h = g_next++;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ivf[h] = iv;
  }
  *out = h;
  return RFX_OK;
}

int rfx_ivf_destroy(rfx_ivf_t h) {
  std::shared_ptr<Ivf> iv;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ivf.find(h);
    if (it == g_ivf.end()) return api_fail(RFX_EINVAL, "unknown IVF handle");
    iv = it->second;
    g_ivf.erase(it);
  }
  IVF_HIP(hipSetDevice(iv->device));
  IVF_HIP(hipDeviceSynchronize());
  return RFX_OK;
}

int rfx_ivf_info(rfx_ivf_t h, int* dim, int* nlist, int64_t* rows, int* trained) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  std::lock_guard<std::mutex> lk(iv->mu);
  if (dim) *dim = iv->dim;
  if (nlist) *nlist = iv->nlist;
  if (rows) *rows = iv->rows;
  if (trained) *trained = iv->trained;
  return RFX_OK;
}

int rfx_quantize(const void* rows_d, int64_t n, int dim, int dtype, int8_t* codes_d, float* inv_d, void* stream) {
  if (n < 0 || dim <= 0 || !valid_dtype(dtype)) return api_fail(RFX_EINVAL, "bad quantize arguments");
  if (n && (!rows_d || !codes_d || !inv_d)) return api_fail(RFX_EINVAL, "null pointers");
  if (n) rfx::ivf::launch_quantize(rows_d, n, dim, dtype, codes_d, inv_d, (hipStream_t)stream);
  IVF_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_synth_clustered(uint64_t cseed, int64_t ncenters, uint64_t seed, int64_t row0, int64_t n, int dim, int dtype,
                        void* out_d, void* stream) {
  if (n < 0 || row0 < 0 || dim <= 0 || ncenters < 1 || !valid_dtype(dtype)) return api_fail(RFX_EINVAL, "bad arguments");
  if (n && !out_d) return api_fail(RFX_EINVAL, "null output");
  if (n) rfx::ivf::launch_synth_clustered(cseed, (uint64_t)ncenters, seed, row0, n, dim, dtype, out_d, (hipStream_t)stream);
  IVF_HIP(hipGetLastError());
  return RFX_OK;
}

int rfx_ivf_train(rfx_ivf_t h, const void* rows_d, int64_t n, int dtype, int iters, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!valid_dtype(dtype) || iters < 0) return api_fail(RFX_EINVAL, "bad dtype / iters");
  std::lock_guard<std::mutex> lk(iv->mu);
  if (n < iv->nlist) return api_fail(RFX_EINVAL, "training needs >= nlist=%d rows (got %lld)", iv->nlist, (long long)n);
  if (!rows_d) return api_fail(RFX_EINVAL, "null rows");
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  const int D = iv->dim, m = iv->nlist;
  uint8_t* tmp = nullptr;
  const size_t bc = al256((size_t)n * D), bi = al256((size_t)n * 4), bs = al256((size_t)m * D * 4), bn = al256((size_t)m * 4);
  if (hipMalloc(&tmp, bc + 2 * bi + bs + bn + al256((size_t)m * 4)) != hipSuccess) return api_fail(RFX_ENOMEM, "hipMalloc failed (train)");
  int8_t* codes = (int8_t*)tmp;
  float* inv = (float*)(tmp + bc);
  int* lab = (int*)(tmp + bc + bi);
  int* sums = (int*)(tmp + bc + 2 * bi);
  int* cnt = (int*)(tmp + bc + 2 * bi + bs);
  int rc = RFX_OK;
  rfx::ivf::launch_quantize(rows_d, n, D, dtype, codes, inv, st);
  // initial centroids: sample rows j * (n / nlist)
  rfx::ivf::launch_init_centroids(codes, n / m, m, D, iv->qc, st);
  rfx::ivf::launch_centroid_update(nullptr, nullptr, m, D, iv->qc, iv->fc, st);
  for (int it = 0; it < iters && rc == RFX_OK; ++it) {
    if (rfx::ivf::launch_assign(codes, n, iv->qc, m, D, iv->fc, lab, nullptr, st)) {
      rc = api_fail(RFX_EUNSUPPORTED, "assignment launch rejected");
      break;
    }
    if (hipMemsetAsync(sums, 0, (size_t)m * D * 4, st) != hipSuccess || hipMemsetAsync(cnt, 0, (size_t)m * 4, st) != hipSuccess) {
      rc = api_fail(RFX_EDEVICE, "memset failed");
      break;
    }
    rfx::ivf::launch_kmeans_accum(codes, n, D, lab, sums, cnt, st);
    rfx::ivf::launch_centroid_update(sums, cnt, m, D, iv->qc, iv->fc, st);
  }
  const hipError_t e = hipStreamSynchronize(st);
  (void)hipFree(tmp);
  if (rc) return rc;
  if (e != hipSuccess) return api_fail(RFX_EDEVICE, "train: %s", hipGetErrorString(e));
  IVF_HIP(hipGetLastError());
  iv->trained = true;
  return assign_all(*iv, 0, iv->rows, st);  // rows added before (re)training move to their new lists
}

int rfx_ivf_set_centroids(rfx_ivf_t h, const int8_t* qc_d, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!qc_d) return api_fail(RFX_EINVAL, "null centroids");
  std::lock_guard<std::mutex> lk(iv->mu);
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  IVF_HIP(hipMemcpyAsync(iv->qc, qc_d, (size_t)iv->nlist * iv->dim, hipMemcpyDeviceToDevice, st));
  rfx::ivf::launch_centroid_update(nullptr, nullptr, iv->nlist, iv->dim, iv->qc, iv->fc, st);
  IVF_HIP(hipGetLastError());
  iv->trained = true;
  return assign_all(*iv, 0, iv->rows, st);
}

int rfx_ivf_get_centroids(rfx_ivf_t h, int8_t* qc_d, float* fc_d, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  std::lock_guard<std::mutex> lk(iv->mu);
  if (!iv->trained) return api_fail(RFX_EINVAL, "IVF index not trained");
  IVF_HIP(hipSetDevice(iv->device));
  if (qc_d) IVF_HIP(hipMemcpyAsync(qc_d, iv->qc, (size_t)iv->nlist * iv->dim, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (fc_d) IVF_HIP(hipMemcpyAsync(fc_d, iv->fc, (size_t)iv->nlist * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return RFX_OK;
}

int rfx_ivf_add(rfx_ivf_t h, const void* rows_d, int64_t n, int dtype, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!valid_dtype(dtype) || n < 0) return api_fail(RFX_EINVAL, "bad dtype / n");
  if (n == 0) return RFX_OK;
  if (!rows_d) return api_fail(RFX_EINVAL, "null rows");
  std::lock_guard<std::mutex> lk(iv->mu);
  if (!iv->trained) return api_fail(RFX_EINVAL, "train the IVF index (or set its centroids) before adding rows");
  if (iv->rows + n >= (int64_t)INT32_MAX) return api_fail(RFX_EUNSUPPORTED, "IVF shard exceeds 2^31-1 rows");
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = grow_rows(*iv, iv->rows + n, st);
  if (rc) return rc;
  rfx::ivf::launch_quantize(rows_d, n, iv->dim, dtype, iv->codes + iv->rows * iv->dim, iv->inv + iv->rows, st);
  const int64_t r0 = iv->rows;
  iv->rows += n;
  return assign_all(*iv, r0, n, st);
}

int rfx_ivf_build(rfx_ivf_t h, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  std::lock_guard<std::mutex> lk(iv->mu);
  IVF_HIP(hipSetDevice(iv->device));
  return build(*iv, (hipStream_t)stream);
}

int rfx_ivf_codes(rfx_ivf_t h, int8_t* codes_d, float* inv_d, int32_t* labels_d, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  std::lock_guard<std::mutex> lk(iv->mu);
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  if (iv->rows == 0) return RFX_OK;
  if (codes_d) IVF_HIP(hipMemcpyAsync(codes_d, iv->codes, (size_t)iv->rows * iv->dim, hipMemcpyDeviceToDevice, st));
  if (inv_d) IVF_HIP(hipMemcpyAsync(inv_d, iv->inv, (size_t)iv->rows * 4, hipMemcpyDeviceToDevice, st));
  if (labels_d) IVF_HIP(hipMemcpyAsync(labels_d, iv->labels, (size_t)iv->rows * 4, hipMemcpyDeviceToDevice, st));
  return RFX_OK;
}

int rfx_ivf_lists(rfx_ivf_t h, int64_t* offsets_d, int32_t* ids_d, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  std::lock_guard<std::mutex> lk(iv->mu);
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = build(*iv, st);
  if (rc) return rc;
  if (offsets_d) IVF_HIP(hipMemcpyAsync(offsets_d, iv->off, (size_t)(iv->nlist + 1) * 8, hipMemcpyDeviceToDevice, st));
  if (ids_d && iv->rows) IVF_HIP(hipMemcpyAsync(ids_d, iv->lids, (size_t)iv->rows * 4, hipMemcpyDeviceToDevice, st));
  return RFX_OK;
}

int rfx_ivf_search_workspace_bytes(rfx_ivf_t h, int64_t nq, int k, int nprobe, size_t* out_bytes) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!out_bytes) return api_fail(RFX_EINVAL, "null out");
  IvfLayout L;
  int rc = ivf_layout(*iv, nq, k, nprobe, L);
  if (rc) return rc;
  *out_bytes = L.total;
  return RFX_OK;
}

int rfx_ivf_search(rfx_ivf_t h, const void* queries_d, int64_t nq, int dtype, int k, int nprobe, float* out_scores_d,
                   int64_t* out_rows_d, void* ws_d, size_t ws_bytes, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!valid_dtype(dtype)) return api_fail(RFX_EINVAL, "bad query dtype");
  IvfLayout L;
  int rc = ivf_layout(*iv, nq, k, nprobe, L);
  if (rc) return rc;
  if (nq == 0) return RFX_OK;
  if (!queries_d || !out_scores_d || !out_rows_d) return api_fail(RFX_EINVAL, "null queries / outputs");
  if (!ws_d || ws_bytes < L.total) return api_fail(RFX_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, L.total);
  std::lock_guard<std::mutex> lk(iv->mu);
  if (!iv->trained) return api_fail(RFX_EINVAL, "IVF index not trained");
  IVF_HIP(hipSetDevice(iv->device));
  hipStream_t st = (hipStream_t)stream;
  if ((rc = build(*iv, st))) return rc;
  uint8_t* ws = (uint8_t*)ws_d;
  int8_t* qq = (int8_t*)(ws + L.qq);
  float* qinv = (float*)(ws + L.qinv);
  float* S = (float*)(ws + L.S);
  int* Sid = (int*)(ws + L.Sid);
  float* ps = (float*)(ws + L.ps);
  int64_t* pid = (int64_t*)(ws + L.pid);
  int* poff = (int*)(ws + L.poff);
  int* pairs = (int*)(ws + L.pairs);
  float* cs = (float*)(ws + L.cs);
  int* cr = (int*)(ws + L.cr);
  rfx::ivf::launch_quantize(queries_d, nq, iv->dim, dtype, qq, qinv, st);
  if (rfx::ivf::launch_coarse_scores(qq, nq, iv->qc, iv->nlist, iv->dim, iv->fc, S, Sid, st))
    return api_fail(RFX_EUNSUPPORTED, "coarse scoring launch rejected");
  if (rfx::ivf::launch_probe_select(S, nq, iv->nlist, nprobe, ps, pid, st) != 0 &&
      rfx::launch_topk_merge(S, Sid, 0, nq, iv->nlist, nprobe, 0, ps, pid, st))
    return api_fail(RFX_EUNSUPPORTED, "probe selection rejected (nprobe=%d)", nprobe);
  if (rfx::ivf::launch_group_pairs(pid, (int)(nq * nprobe), iv->nlist, poff, pairs, st))
    return api_fail(RFX_EUNSUPPORTED, "pair grouping rejected");
  if (rfx::ivf::launch_list_scan(L.K, iv->dim, iv->nlist, L.splits, iv->lcodes, iv->linv, iv->lids, iv->off, poff, pairs, nprobe,
                                 qq, qinv, cs, cr, st))
    return api_fail(RFX_EUNSUPPORTED, "list scan launch rejected (k=%d dim=%d)", k, iv->dim);
  // (the wave lists are sorted best first, empty slots last: the merge reads each only as far as it can
  // still admit)
  if (rfx::launch_topk_merge_lists(cs, cr, 0, nq, L.ncand, L.K, k, 0, out_scores_d, out_rows_d, nullptr, st,
                                   /*sorted=*/true))
    return api_fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  IVF_HIP(hipGetLastError());
  return RFX_OK;
}

// Search with exact re-rank: the IVF search keeps rerank_k (>= k) candidates per query by int8
// score, then every candidate is re-scored against its original row (rows_d: [rows][dim] of
// rows_dtype in insertion order, e.g. rfx_index_data of the brute-force store holding the same
// rows) in f32, and the merge keeps the top k.  Workspace: rfx_ivf_rerank_workspace_bytes.
int rfx_ivf_rerank_workspace_bytes(rfx_ivf_t h, int64_t nq, int k, int nprobe, int rerank_k, size_t* out_bytes) {
  if (rerank_k < k || rerank_k > 64) return api_fail(RFX_EINVAL, "rerank_k=%d must be in [k=%d, 64]", rerank_k, k);
  size_t ivf = 0;
  int rc = rfx_ivf_search_workspace_bytes(h, nq, rerank_k, nprobe, &ivf);
  if (rc) return rc;
  if (!out_bytes) return api_fail(RFX_EINVAL, "null out");
  *out_bytes = al256(ivf) + 3 * al256((size_t)nq * rerank_k * 8);
  return RFX_OK;
}

int rfx_ivf_search_rerank(rfx_ivf_t h, const void* queries_d, int64_t nq, int dtype, int k, int nprobe, int rerank_k,
                          const void* rows_d, int rows_dtype, float* out_scores_d, int64_t* out_rows_d, void* ws_d,
                          size_t ws_bytes, void* stream) {
  auto iv = get(h);
  if (!iv) return api_fail(RFX_EINVAL, "unknown IVF handle");
  if (!valid_dtype(rows_dtype) || !valid_dtype(dtype)) return api_fail(RFX_EINVAL, "bad dtype");
  size_t need = 0, ivf = 0;
  int rc = rfx_ivf_rerank_workspace_bytes(h, nq, k, nprobe, rerank_k, &need);
  if (rc) return rc;
  if (nq == 0) return RFX_OK;
  if (!rows_d || !queries_d || !out_scores_d || !out_rows_d) return api_fail(RFX_EINVAL, "null pointers");
  if (!ws_d || ws_bytes < need) return api_fail(RFX_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, need);
  rfx_ivf_search_workspace_bytes(h, nq, rerank_k, nprobe, &ivf);
  uint8_t* ws = (uint8_t*)ws_d;
  float* cs = (float*)(ws + al256(ivf));
  int64_t* cr = (int64_t*)(ws + al256(ivf) + al256((size_t)nq * rerank_k * 8));
  float* rs = (float*)(ws + al256(ivf) + 2 * al256((size_t)nq * rerank_k * 8));
  int64_t* rr = cr;  // the re-rank kernel rewrites rows in place (padding -> empty sentinel)
  if ((rc = rfx_ivf_search(h, queries_d, nq, dtype, rerank_k, nprobe, cs, cr, ws, al256(ivf), stream))) return rc;
  hipStream_t st = (hipStream_t)stream;
  IVF_HIP(hipSetDevice(iv->device));
  if (rfx::ivf::launch_rerank(queries_d, dtype, rows_d, rows_dtype, iv->dim, cr, nq, rerank_k, rs, rr, st))
    return api_fail(RFX_EUNSUPPORTED, "re-rank launch rejected");
  if (rfx::launch_topk_merge(rs, rr, 1, nq, rerank_k, k, 0, out_scores_d, out_rows_d, st))
    return api_fail(RFX_EUNSUPPORTED, "merge k=%d unsupported", k);
  IVF_HIP(hipGetLastError());
  return RFX_OK;
}

// The re-rank step alone over one shard's rows (rfx/sharded.py ShardedIvf): candidates are global
// rows, the shard owns [row_lo, row_lo + n_rows).  The same kernel as rfx_ivf_search_rerank.
int rfx_rerank_candidates(const void* queries_d, int64_t nq, int dtype, const void* rows_d, int rows_dtype,
                          int64_t row_lo, int64_t n_rows, int dim, const int64_t* cand_d, int n_cand,
                          float* out_scores_d, int64_t* out_rows_d, void* stream) {
  if (!valid_dtype(rows_dtype) || !valid_dtype(dtype)) return api_fail(RFX_EINVAL, "bad dtype");
  if (nq < 0 || n_cand < 0 || dim <= 0 || row_lo < 0 || n_rows < 0)
    return api_fail(RFX_EINVAL, "bad sizes (nq %lld, n_cand %d, dim %d, rows [%lld, +%lld))", (long long)nq, n_cand,
                    dim, (long long)row_lo, (long long)n_rows);
  if (nq == 0 || n_cand == 0) return RFX_OK;
  if (!queries_d || !cand_d || !out_scores_d || !out_rows_d || (n_rows > 0 && !rows_d))
    return api_fail(RFX_EINVAL, "null pointers");
  hipStream_t st = (hipStream_t)stream;
  if (rfx::ivf::launch_rerank(queries_d, dtype, rows_d, rows_dtype, dim, cand_d, nq, n_cand, out_scores_d, out_rows_d,
                              st, row_lo, n_rows))
    return api_fail(RFX_EUNSUPPORTED, "re-rank launch rejected");
  IVF_HIP(hipGetLastError());
  return RFX_OK;
}

// Persistence: "RFXIVF01", {version 1, dim, nlist, trained}, rows, then the int8 centroids and
// the per-row codes / scales / labels in insertion order.  Factors and posting lists are derived
// (recomputed on load).  Written to path.tmp, then renamed.
int rfx_ivf_save(rfx_ivf_t h, const char* path) {
  auto iv = get(h);
  if (!iv || !path) return api_fail(RFX_EINVAL, "unknown IVF handle / null path");
  std::lock_guard<std::mutex> lk(iv->mu);
  IVF_HIP(hipSetDevice(iv->device));
  IVF_HIP(hipDeviceSynchronize());
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return api_fail(RFX_EIO, "cannot open %s", tmp.c_str());
  const uint32_t hdr[4] = {1u, (uint32_t)iv->dim, (uint32_t)iv->nlist, (uint32_t)iv->trained};
  const int64_t rows = iv->rows;
  bool ok = fwrite("RFXIVF01", 1, 8, f) == 8 && fwrite(hdr, 4, 4, f) == 4 && fwrite(&rows, 8, 1, f) == 1;
  ok = ok && write_dev(f, iv->qc, (size_t)iv->nlist * iv->dim);
  if (rows > 0) {
    ok = ok && write_dev(f, iv->codes, (size_t)rows * iv->dim) && write_dev(f, iv->inv, (size_t)rows * 4) &&
         write_dev(f, iv->labels, (size_t)rows * 4);
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok) return api_fail(RFX_EIO, "write failed for %s", tmp.c_str());
  if (rename(tmp.c_str(), path) != 0) return api_fail(RFX_EIO, "rename to %s failed", path);
  return RFX_OK;
}

int rfx_ivf_load(const char* path, int device, rfx_ivf_t* out) {
  if (!path || !out) return api_fail(RFX_EINVAL, "null path / out");
  FILE* f = fopen(path, "rb");
  if (!f) return api_fail(RFX_EIO, "cannot open %s", path);
  char magic[8];
  uint32_t hdr[4];
  int64_t rows = 0;
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "RFXIVF01", 8) != 0 || fread(hdr, 4, 4, f) != 4 ||
      fread(&rows, 8, 1, f) != 1 || hdr[0] != 1u || rows < 0) {
    fclose(f);
    return api_fail(RFX_EIO, "%s is not an rfx IVF file", path);
  }
  rfx_ivf_t h = 0;
  int rc = rfx_ivf_create(device, (int)hdr[1], (int)hdr[2], &h);
  if (rc) {
    fclose(f);
    return rc;
  }
  auto iv = get(h);
  bool ok = read_dev(f, iv->qc, (size_t)iv->nlist * iv->dim);
  if (ok && rows > 0) {
    rc = grow_rows(*iv, rows, nullptr);
    ok = rc == RFX_OK && read_dev(f, iv->codes, (size_t)rows * iv->dim) && read_dev(f, iv->inv, (size_t)rows * 4) &&
         read_dev(f, iv->labels, (size_t)rows * 4);
  }
  fclose(f);
  if (!ok) {
    rfx_ivf_destroy(h);
    return rc ? rc : api_fail(RFX_EIO, "truncated IVF file %s", path);
  }
  iv->rows = rows;
  iv->trained = hdr[3] != 0;
  iv->dirty = true;
  rfx::ivf::launch_centroid_update(nullptr, nullptr, iv->nlist, iv->dim, iv->qc, iv->fc, nullptr);
  IVF_HIP(hipDeviceSynchronize());
  *out = h;
  return RFX_OK;
}

}  // extern "C"
