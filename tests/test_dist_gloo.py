"""CPU, world_size 2 (gloo): the multi-GPU exchange step of rfx.dist — row partition, packed
all-gather of per-shard top-k, merge — equals the unsharded oracle top-k."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rfx import dist as rdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_merge(cs, cr, k):
    """Test-side merge (the GPU path uses the HIP kernel rfx.index.topk_merge)."""
    s = cs.numpy().astype(np.float64)
    r = cr.numpy()
    out_s = np.full((s.shape[0], k), -np.inf, dtype=np.float32)
    out_r = np.full((s.shape[0], k), -1, dtype=np.int64)
    for i in range(s.shape[0]):
        live = r[i] >= 0
        order = np.lexsort((r[i][live], -s[i][live]))[:k]
        out_s[i, :len(order)] = s[i][live][order]
        out_r[i, :len(order)] = r[i][live][order]
    return torch.from_numpy(out_s), torch.from_numpy(out_r)


def _worker(rank, world, port, n_rows, nq, k, result):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import search, synth
    r0, r1 = rdist.shard_range(n_rows, rank, world)
    rows = synth.to_f64(synth.synth_rows(5, r0, r1 - r0, 64, "bf16"), "bf16")  # generator rows = global ids
    q = synth.to_f64(synth.synth_rows(6, 0, nq, 64, "bf16"), "bf16")
    ls, lr = search.topk(q, rows, k)
    lr = np.where(lr >= 0, lr + r0, lr)
    s, r = rdist.gather_merge(torch.from_numpy(ls.astype(np.float32)), torch.from_numpy(lr), k, _oracle_merge)
    if rank == 0:
        result.put((s.numpy(), r.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_rows", [(2, 3001), (3, 100), (2, 3)])
def test_sharded_search_equals_whole(world, n_rows):
    from oracle import search, synth
    nq, k = 5, 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _free_port(), n_rows, nq, k, q), nprocs=world, start_method="spawn")
    s, r = q.get(timeout=60)
    rows = synth.to_f64(synth.synth_rows(5, 0, n_rows, 64, "bf16"), "bf16")
    qq = synth.to_f64(synth.synth_rows(6, 0, nq, 64, "bf16"), "bf16")
    ref_s, ref_r = search.topk(qq, rows, k)
    assert np.array_equal(r, ref_r)
    live = ref_r >= 0
    assert np.allclose(s[live], ref_s[live], atol=1e-6)


def test_shard_range_partition():
    for n in (0, 1, 7, 10_000_000, 100_000_001):
        for w in (1, 2, 3, 8):
            spans = [rdist.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_roundtrip():
    s = torch.tensor([[0.5, -0.25, float("-inf")], [1.0, 0.0, -1.0]])
    r = torch.tensor([[3, 9, -1], [0, 2 ** 40, 5]])
    packed = torch.stack([rdist.pack(s, r), rdist.pack(s * 2, r + 1)])  # world of 2
    cs, cr = rdist.unpack(packed)
    assert torch.equal(cs[:, :3], s) and torch.equal(cr[:, 3:], r + 1)
