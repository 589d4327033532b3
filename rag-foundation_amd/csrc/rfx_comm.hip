// rfx_comm.hip — the multi-GPU exchange of the retrieval path inside the C ABI: RCCL
// communicators and the all-gather of per-shard partial top-k records over xGMI.
//
// The reference has no collective of any kind; this is the one exchange step the
// row-sharded corpus needs.  Two process models (SURVEY §8e, §7 "Process topology"):
//   * one process per GPU: rank 0 makes an ncclUniqueId (rfx_comm_unique_id), the host hands it to
//     the other ranks once (bootstrap only, e.g. torch.distributed's store), each rank calls
//     rfx_comm_init_rank;
//   * one index-server process owning several GPUs: rfx_comm_init_all (ncclCommInitAll), and the
//     all-gather runs as one RCCL group over the process's devices.
// The payload is tiny (nq·k·16 B per rank: 40 KB at nq 256, k 10), so the collective is latency-
// bound over xGMI; one ncclAllGather per batch, no bucketing — or, where only one rank assembles the
// answer (the query's front end), rfx_gather_records: grouped ncclSend / ncclRecv to that rank, one
// hop over the point-to-point links.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "rfx_kernels.h"

namespace {

struct Comm {
  std::vector<ncclComm_t> comms;  // one per local device (rank mode: exactly one)
  std::vector<int> devices;
  int world = 0;
  int rank = 0;  // rank mode: this process's rank; group mode: 0
  bool group = false;
  // One communicator must see its collectives in the same order on every device.  Searches of
  // different (store, filter) batches run in parallel threads against one ShardedIndex, so the
  // group start .. end of one all-gather is made atomic here.
  std::mutex mu;
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<Comm>> g_comms;
uint64_t g_next = 1;

std::shared_ptr<Comm> get(rfx_comm_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(h);
  return it == g_comms.end() ? nullptr : it->second;
}

rfx_comm_t put(std::shared_ptr<Comm> c) {
  std::lock_guard<std::mutex> lk(g_mu);
  const uint64_t h = g_next++;
  g_comms[h] = std::move(c);
  return h;
}

#define RFX_NCCL(call)                                                                                \
  do {                                                                                                \
    ncclResult_t r_ = (call);                                                                         \
    if (r_ != ncclSuccess) return rfx::api_fail(RFX_EDEVICE, "%s: %s", #call, ncclGetErrorString(r_)); \
  } while (0)

}  // namespace

static_assert(sizeof(ncclUniqueId) == RFX_COMM_ID_BYTES, "ncclUniqueId size");

extern "C" {

int rfx_comm_unique_id(void* out_id) {
  if (!out_id) return rfx::api_fail(RFX_EINVAL, "null out");
  ncclUniqueId id;
  RFX_NCCL(ncclGetUniqueId(&id));
  memcpy(out_id, &id, sizeof(id));
  return RFX_OK;
}

int rfx_comm_init_rank(int world, int rank, const void* unique_id, int device, rfx_comm_t* out) {
  if (!unique_id || !out) return rfx::api_fail(RFX_EINVAL, "null id / out");
  if (world < 1 || rank < 0 || rank >= world) return rfx::api_fail(RFX_EINVAL, "rank %d of world %d", rank, world);
  if (hipSetDevice(device) != hipSuccess) return rfx::api_fail(RFX_EDEVICE, "hipSetDevice(%d)", device);
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  auto c = std::make_shared<Comm>();
  c->comms.resize(1);
  RFX_NCCL(ncclCommInitRank(&c->comms[0], world, id, rank));
  c->devices = {device};
  c->world = world;
  c->rank = rank;
  *out = put(c);
  return RFX_OK;
}

int rfx_comm_init_all(int n, const int* device_ids, rfx_comm_t* out) {
  if (n < 1 || !device_ids || !out) return rfx::api_fail(RFX_EINVAL, "n < 1 / null arguments");
  auto c = std::make_shared<Comm>();
  c->comms.resize(n);
  RFX_NCCL(ncclCommInitAll(c->comms.data(), n, device_ids));
  c->devices.assign(device_ids, device_ids + n);
  c->world = n;
  c->group = true;
  *out = put(c);
  return RFX_OK;
}

int rfx_comm_info(rfx_comm_t h, int* world, int* rank, int* n_local) {
  auto c = get(h);
  if (!c) return rfx::api_fail(RFX_EINVAL, "unknown communicator");
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  if (n_local) *n_local = (int)c->comms.size();
  return RFX_OK;
}

int rfx_comm_destroy(rfx_comm_t h) {
  std::shared_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(h);
    if (it == g_comms.end()) return rfx::api_fail(RFX_EINVAL, "unknown communicator");
    c = it->second;
    g_comms.erase(it);
  }
  std::lock_guard<std::mutex> lk(c->mu);  // no all-gather of another thread is mid-enqueue
  for (auto& cm : c->comms) RFX_NCCL(ncclCommDestroy(cm));
  return RFX_OK;
}

int rfx_allgather_records(rfx_comm_t h, const void* const* sends_d, void* const* recvs_d, int64_t nq, int k,
                          void* const* streams) {
  auto c = get(h);
  if (!c) return rfx::api_fail(RFX_EINVAL, "unknown communicator");
  if (nq < 0 || k < 1 || k > 64) return rfx::api_fail(RFX_EINVAL, "nq %lld, k %d", (long long)nq, k);
  if (!sends_d || !recvs_d || !streams) return rfx::api_fail(RFX_EINVAL, "null buffer arrays");
  const size_t bytes = (size_t)nq * k * 16;  // {f32 score, i32 pad, i64 row} records
  if (bytes == 0) return RFX_OK;
  const int n = (int)c->comms.size();
  for (int i = 0; i < n; ++i)
    if (!sends_d[i] || !recvs_d[i]) return rfx::api_fail(RFX_EINVAL, "null buffer for local device %d", i);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return rfx::api_fail(RFX_EDEVICE, "hipGetDevice");
  std::lock_guard<std::mutex> lk(c->mu);
  if (n > 1) RFX_NCCL(ncclGroupStart());
  int rc = RFX_OK;
  for (int i = 0; i < n && rc == RFX_OK; ++i) {
    if (hipSetDevice(c->devices[i]) != hipSuccess) {
      rc = rfx::api_fail(RFX_EDEVICE, "hipSetDevice(%d)", c->devices[i]);
      break;
    }
    const ncclResult_t r = ncclAllGather(sends_d[i], recvs_d[i], bytes, ncclUint8, c->comms[i], (hipStream_t)streams[i]);
    if (r != ncclSuccess) rc = rfx::api_fail(RFX_EDEVICE, "ncclAllGather: %s", ncclGetErrorString(r));
  }
  if (n > 1) {
    const ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess && rc == RFX_OK) rc = rfx::api_fail(RFX_EDEVICE, "ncclGroupEnd: %s", ncclGetErrorString(r));
  }
  (void)hipSetDevice(prev);
  return rc;
}

int rfx_gather_records(rfx_comm_t h, const void* const* sends_d, void* const* recvs_d, int root, int64_t nq, int k,
                       void* const* streams) {
  auto c = get(h);
  if (!c) return rfx::api_fail(RFX_EINVAL, "unknown communicator");
  if (nq < 0 || k < 1 || k > 64) return rfx::api_fail(RFX_EINVAL, "nq %lld, k %d", (long long)nq, k);
  if (root < 0 || root >= c->world) return rfx::api_fail(RFX_EINVAL, "root %d of world %d", root, c->world);
  if (!sends_d || !recvs_d || !streams) return rfx::api_fail(RFX_EINVAL, "null buffer arrays");
  const size_t bytes = (size_t)nq * k * 16;
  if (bytes == 0) return RFX_OK;
  const int n = (int)c->comms.size();
  // the local index of the root (group mode: device index root; rank mode: 0 when this rank is root)
  const int lroot = c->group ? root : (c->rank == root ? 0 : -1);
  for (int i = 0; i < n; ++i)
    if (!sends_d[i] || (i == lroot && !recvs_d[i]))
      return rfx::api_fail(RFX_EINVAL, "null buffer for local device %d", i);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return rfx::api_fail(RFX_EDEVICE, "hipGetDevice");
  std::lock_guard<std::mutex> lk(c->mu);
  RFX_NCCL(ncclGroupStart());
  int rc = RFX_OK;
  for (int i = 0; i < n && rc == RFX_OK; ++i) {
    if (hipSetDevice(c->devices[i]) != hipSuccess) {
      rc = rfx::api_fail(RFX_EDEVICE, "hipSetDevice(%d)", c->devices[i]);
      break;
    }
    hipStream_t st = (hipStream_t)streams[i];
    if (i == lroot)
      for (int p = 0; p < c->world && rc == RFX_OK; ++p) {
        const ncclResult_t r = ncclRecv((uint8_t*)recvs_d[i] + (size_t)p * bytes, bytes, ncclUint8, p, c->comms[i], st);
        if (r != ncclSuccess) rc = rfx::api_fail(RFX_EDEVICE, "ncclRecv from %d: %s", p, ncclGetErrorString(r));
      }
    if (rc != RFX_OK) break;
    const ncclResult_t r = ncclSend(sends_d[i], bytes, ncclUint8, root, c->comms[i], st);
    if (r != ncclSuccess) rc = rfx::api_fail(RFX_EDEVICE, "ncclSend: %s", ncclGetErrorString(r));
  }
  const ncclResult_t r = ncclGroupEnd();
  if (r != ncclSuccess && rc == RFX_OK) rc = rfx::api_fail(RFX_EDEVICE, "ncclGroupEnd: %s", ncclGetErrorString(r));
  (void)hipSetDevice(prev);
  return rc;
}

}  // extern "C"
