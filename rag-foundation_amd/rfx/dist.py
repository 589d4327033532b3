"""Row-sharded multi-GPU search: one process per GPU, torch.distributed (backend "nccl" = RCCL
over xGMI on ROCm).

Partition: rank r owns global rows [offset_r, offset_r + n_r) (contiguous ranges, as even as
possible).  Per batch every rank (1) scans its shard into a local top-k, (2) adds its row offset,
(3) all-gathers the packed (score, row) lists — nq·k·16 B per rank, latency-bound on xGMI —
and (4) merges the world_size·k candidates per query with the same ranking rule.  This is the
only collective on the path; the reference has none.
"""
import torch
import torch.distributed as dist


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


def gather_merge(local_s: torch.Tensor, local_r: torch.Tensor, k: int, merge, group=None):
    """All-gather every rank's local top-k (rows already global) and merge them.

    `merge(cand_scores, cand_rows, k)` is the HIP top-k merge (rfx.index.topk_merge) on the GPU
    path; the gloo CPU tests pass their own.  Returns the global (scores, rows) on every rank.
    """
    world = dist.get_world_size(group)
    if world == 1:
        return local_s, local_r
    mine = pack(local_s, local_r)
    out = torch.empty((world * mine.shape[0],) + tuple(mine.shape[1:]), dtype=mine.dtype, device=mine.device)
    dist.all_gather_into_tensor(out, mine, group=group)  # ranks concatenated along dim 0
    cs, cr = unpack(out.view((world,) + tuple(mine.shape)))
    return merge(cs, cr, k)


def gather_merge_records(records: torch.Tensor, k: int, group=None, stream=None):
    """GPU path: all-gather this rank's [nq][k][2] int64 records (rfx.index.topk_merge_records,
    rows already global) and merge the world's records with the HIP kernel.  Two device ops and
    one collective per batch; no host-side tensor reshuffling."""
    from .index import merge_gathered

    world = dist.get_world_size(group)
    if world == 1:
        return merge_gathered(records.unsqueeze(0), k, stream=stream)
    if dist.get_backend(group) == "gloo":
        # gloo moves host tensors (tests / hosts without RCCL): the exchange goes through host
        # memory, the merge still runs on the device
        parts = [torch.empty_like(records, device="cpu") for _ in range(world)]
        dist.all_gather(parts, records.cpu(), group=group)
        return merge_gathered(torch.stack(parts).to(records.device), k, stream=stream)
    out = torch.empty((world,) + tuple(records.shape), dtype=records.dtype, device=records.device)
    dist.all_gather_into_tensor(out, records, group=group)  # RCCL over xGMI; ranks along dim 0
    return merge_gathered(out, k, stream=stream)


class ShardedSearch:
    """Holds this rank's DeviceIndex shard and runs the global search."""

    def __init__(self, index, row_offset: int, group=None):
        self.index = index
        self.row_offset = int(row_offset)
        self.group = group

    def search(self, queries: torch.Tensor, k: int, workspace=None, stream=None):
        from .index import topk_merge_records

        cs, cr = self.index.scan(queries, k, workspace=workspace, stream=stream)
        rec = topk_merge_records(cs, cr, k, row_offset=self.row_offset, stream=stream,
                                 list_len=self.index.list_len(queries.shape[0], k))
        return gather_merge_records(rec, k, self.group, stream=stream)


class ShardedIvf:
    """Row-sharded IVF-Flat int8: every rank holds its rows' part of every
    posting list under ONE coarse quantiser.  Rank 0 trains k-means on its sample and the int8
    centroids are broadcast (nlist·dim bytes, once); each rank quantises/assigns its own rows.
    A search is the brute-force path's exchange: local IVF top-k -> records with the rank's row
    offset -> one all-gather -> rfx_merge_gathered."""

    def __init__(self, ivf, row_offset: int, group=None):
        self.ivf = ivf
        self.row_offset = int(row_offset)
        self.group = group

    def train(self, sample: torch.Tensor = None, iters: int = 10, src: int = 0):
        """Rank `src` trains on `sample`; the centroids reach every rank by broadcast."""
        if dist.get_rank(self.group) == src:
            self.ivf.train(sample, iters=iters)
            qc = self.ivf.centroids()[0]
        else:
            qc = torch.empty((self.ivf.nlist, self.ivf.dim), dtype=torch.int8, device=self.ivf._dev())
        if dist.get_world_size(self.group) > 1:
            if dist.get_backend(self.group) == "gloo":
                host = qc.cpu()
                dist.broadcast(host, src=src, group=self.group)
                qc = host.to(qc.device)
            else:
                dist.broadcast(qc, src=src, group=self.group)
        if dist.get_rank(self.group) != src:
            self.ivf.set_centroids(qc)

    def search(self, queries: torch.Tensor, k: int, nprobe: int, workspace=None, stream=None):
        from .index import topk_merge_records

        s, r = self.ivf.search(queries, k, nprobe, workspace=workspace, stream=stream)
        rec = topk_merge_records(s, r, k, row_offset=self.row_offset, stream=stream)
        return gather_merge_records(rec, k, self.group, stream=stream)
