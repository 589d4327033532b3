"""Row-sharded multi-GPU search: the corpus is split into contiguous row ranges, one
per GPU; every batch each shard scans its rows into a local top-k, adds its row offset, the
shards' packed (score, row) records are all-gathered — nq·k·16 B per shard, latency-bound on
xGMI — and merged with the same ranking rule.  This is the only collective on the path; the
reference has none.

The collective runs inside librfx on RCCL (rfx_comm_* / rfx_allgather_records, include/rfx.h);
the host only bootstraps the communicator:
  * one process per GPU (bench.py --gpus N under torch.distributed.run): RcclComm.for_rank —
    rank 0 makes the 128-byte id, torch.distributed hands it to the other ranks once;
  * one process owning several GPUs (an index-server API process, rfx.sharded.ShardedIndex):
    RcclComm.for_devices (ncclCommInitAll), one RCCL group over the process's devices.
Without an RCCL communicator (gloo process group: CPU tests, multi-rank rehearsal on one GPU) the
records travel through host memory instead; the merge is the same HIP kernel.
"""
import ctypes

import torch
import torch.distributed as dist

from ._lib import check, lib

ID_BYTES = 128  # RFX_COMM_ID_BYTES


def shard_range(n_rows: int, rank: int, world: int):
    """[start, end) of rank's contiguous share of n_rows."""
    base, extra = divmod(n_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack(scores: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """[nq][k] f32 scores + int64 rows -> one [nq][k][2] int64 buffer (one collective)."""
    return torch.stack([scores.contiguous().view(torch.int32).to(torch.int64), rows], dim=-1)


def unpack(packed: torch.Tensor):
    """[world][nq][k][2] -> (scores [nq][world*k] f32, rows [nq][world*k] int64)."""
    world, nq, k, _ = packed.shape
    p = packed.permute(1, 0, 2, 3).reshape(nq, world * k, 2)
    scores = p[..., 0].to(torch.int32).contiguous().view(torch.float32)
    return scores, p[..., 1].contiguous()


class RcclComm:
    """An RCCL communicator owned by librfx (rfx_comm_t)."""

    def __init__(self, handle: int, devices):
        self.handle = handle
        self.devices = list(devices)
        w, r, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.rfx_comm_info(handle, ctypes.byref(w), ctypes.byref(r), ctypes.byref(n)))
        self.world, self.rank, self.n_local = w.value, r.value, n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(ID_BYTES)
        check(lib.rfx_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def for_rank(cls, world: int, rank: int, device: int, unique_id: bytes) -> "RcclComm":
        if len(unique_id) != ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        h = ctypes.c_uint64()
        with torch.cuda.device(device):
            check(lib.rfx_comm_init_rank(int(world), int(rank), ctypes.c_char_p(unique_id), int(device), ctypes.byref(h)))
        return cls(h.value, [device])

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "RcclComm":
        """Bootstrap over an initialised torch.distributed group (any backend): rank 0's id is
        broadcast once; nothing of the data path goes through torch.distributed."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls.for_rank(world, rank, device, obj[0])

    @classmethod
    def for_devices(cls, devices) -> "RcclComm":
        devs = [int(d) for d in devices]
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_uint64()
        check(lib.rfx_comm_init_all(len(devs), arr, ctypes.byref(h)))
        return cls(h.value, devs)

    def allgather_records(self, sends, recvs, streams):
        """sends[i]: [nq][k][2] int64 records on local device i; recvs[i]: [world][nq][k][2]."""
        n = self.n_local
        if not (len(sends) == len(recvs) == len(streams) == n):
            raise ValueError(f"need {n} send/recv/stream entries")
        nq, k = sends[0].shape[0], sends[0].shape[1]
        for s, r in zip(sends, recvs):
            if s.shape != (nq, k, 2) or r.shape != (self.world, nq, k, 2) or s.dtype != torch.int64 \
                    or r.dtype != torch.int64 or not (s.is_contiguous() and r.is_contiguous()):
                raise ValueError("records must be contiguous int64 [nq][k][2] -> [world][nq][k][2]")
        sp = (ctypes.c_void_p * n)(*[s.data_ptr() for s in sends])
        rp = (ctypes.c_void_p * n)(*[r.data_ptr() for r in recvs])
        stp = (ctypes.c_void_p * n)(*[st.cuda_stream for st in streams])
        check(lib.rfx_allgather_records(self.handle, sp, rp, nq, k, stp))

    def gather_records(self, sends, recvs, streams, root: int = 0):
        """sends[i]: [nq][k][2] int64 records on local device i; recvs[i]: [world][nq][k][2] on the
        local device that is `root` (None elsewhere): grouped send / recv to one rank."""
        n = self.n_local
        if not (len(sends) == len(recvs) == len(streams) == n):
            raise ValueError(f"need {n} send/recv/stream entries")
        nq, k = sends[0].shape[0], sends[0].shape[1]
        lroot = root if self.n_local > 1 else (0 if self.rank == root else -1)
        for i, (s, r) in enumerate(zip(sends, recvs)):
            if s.shape != (nq, k, 2) or s.dtype != torch.int64 or not s.is_contiguous():
                raise ValueError("records must be contiguous int64 [nq][k][2]")
            if i == lroot and (r is None or r.shape != (self.world, nq, k, 2) or r.dtype != torch.int64
                               or not r.is_contiguous()):
                raise ValueError("the root's receive buffer must be contiguous int64 [world][nq][k][2]")
        sp = (ctypes.c_void_p * n)(*[s.data_ptr() for s in sends])
        rp = (ctypes.c_void_p * n)(*[r.data_ptr() if r is not None else None for r in recvs])
        stp = (ctypes.c_void_p * n)(*[st.cuda_stream for st in streams])
        check(lib.rfx_gather_records(self.handle, sp, rp, int(root), nq, k, stp))

    def close(self):
        if getattr(self, "handle", None):
            check(lib.rfx_comm_destroy(self.handle))
            self.handle = None


def gather_merge(local_s: torch.Tensor, local_r: torch.Tensor, k: int, merge, group=None):
    """Host-tensor exchange (gloo; CPU tests): all-gather every rank's local top-k (rows already
    global) and merge them with `merge(cand_scores, cand_rows, k)`."""
    world = dist.get_world_size(group)
    if world == 1:
        return local_s, local_r
    mine = pack(local_s, local_r)
    out = torch.empty((world * mine.shape[0],) + tuple(mine.shape[1:]), dtype=mine.dtype, device=mine.device)
    dist.all_gather_into_tensor(out, mine, group=group)  # ranks concatenated along dim 0
    cs, cr = unpack(out.view((world,) + tuple(mine.shape)))
    return merge(cs, cr, k)


def gather_merge_records(records: torch.Tensor, k: int, comm: RcclComm = None, group=None, stream=None):
    """All-gather this rank's [nq][k][2] records (rfx.index.topk_merge_records, rows already
    global) and merge the world's records with the HIP kernel, all on `stream` (default: the
    current stream): records -> RCCL all-gather -> rfx_merge_gathered are ordered by the stream."""
    from .index import merge_gathered

    stream = stream if stream is not None else torch.cuda.current_stream(records.device)
    if comm is not None:
        out = torch.empty((comm.world,) + tuple(records.shape), dtype=records.dtype, device=records.device)
        comm.allgather_records([records], [out], [stream])
        return merge_gathered(out, k, stream=stream)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return merge_gathered(records.unsqueeze(0), k, stream=stream)
    # no RCCL communicator (gloo group: rehearsal of N ranks sharing one GPU): via host memory
    with torch.cuda.stream(stream):
        host = records.cpu()  # ordered after the records' producer on `stream`
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        gathered = torch.stack(parts).to(records.device)
    return merge_gathered(gathered, k, stream=stream)


class ShardedSearch:
    """Holds this rank's DeviceIndex shard and runs the global search."""

    def __init__(self, index, row_offset: int, comm: RcclComm = None, group=None):
        self.index = index
        self.row_offset = int(row_offset)
        self.comm = comm
        self.group = group

    def search(self, queries: torch.Tensor, k: int, workspace=None, stream=None, row_mask=None):
        """This rank's whole search as records (rfx_search_records: the exact two-pass scan when the
        shard holds its int8 copy, the exact scan + merge otherwise; rows + row_offset), then the
        exchange and the gathered merge."""
        rec = self.index.search_records(queries, k, row_offset=self.row_offset, workspace=workspace, stream=stream,
                                        row_mask=row_mask)
        return gather_merge_records(rec, k, self.comm, self.group, stream=stream)


class ShardedIvf:
    """Row-sharded IVF-Flat int8: every rank holds its rows' part of every
    posting list under ONE coarse quantiser.  Rank 0 trains k-means on its sample and the int8
    centroids are broadcast (nlist·dim bytes, once, at build time); each rank quantises/assigns
    its own rows.  A search is the brute-force path's exchange: local IVF top-k -> records with the
    rank's row offset -> one all-gather -> rfx_merge_gathered."""

    def __init__(self, ivf, row_offset: int, comm: RcclComm = None, group=None):
        self.ivf = ivf
        self.row_offset = int(row_offset)
        self.comm = comm
        self.group = group

    def train(self, sample: torch.Tensor = None, iters: int = 10, src: int = 0):
        """Rank `src` trains on `sample`; the centroids reach every rank by broadcast (build time,
        not the search path)."""
        if dist.get_rank(self.group) == src:
            self.ivf.train(sample, iters=iters)
            qc = self.ivf.centroids()[0]
        else:
            qc = torch.empty((self.ivf.nlist, self.ivf.dim), dtype=torch.int8, device=self.ivf._dev())
        if dist.get_world_size(self.group) > 1:
            host = qc.cpu()
            dist.broadcast(host, src=src, group=self.group)
            qc = host.to(qc.device)
        if dist.get_rank(self.group) != src:
            self.ivf.set_centroids(qc)

    def search(self, queries: torch.Tensor, k: int, nprobe: int, workspace=None, stream=None):
        from .index import topk_merge_records

        s, r = self.ivf.search(queries, k, nprobe, workspace=workspace, stream=stream)
        rec = topk_merge_records(s, r, k, row_offset=self.row_offset, stream=stream)
        return gather_merge_records(rec, k, self.comm, self.group, stream=stream)

