"""GPU, world_size 2 on one device (gloo transport): the multi-GPU step of rfx.dist — per-rank
scan of a row shard, rfx_topk_merge_records, all-gather, rfx_merge_gathered — equals the
single-index search of the whole corpus.  (The 8-GPU RCCL run is the driver's; this pins the
exchange logic and the HIP kernels around it.)"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, nq, k, dtype, result):
    import torch.distributed as dist

    from rfx import dist as rdist
    from rfx.index import DeviceIndex, synth_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    r0, r1 = rdist.shard_range(n, rank, world)
    ix = DeviceIndex(768, dtype, 0)
    ix.add_synthetic(31, r1 - r0, gen_row0=r0)
    q = synth_rows(32, 0, nq, 768, dtype)
    s, r = rdist.ShardedSearch(ix, r0).search(q, k)
    if rank == 0:
        full = DeviceIndex(768, dtype, 0)
        full.add_synthetic(31, n)
        fs, fr = full.search(q, k)
        torch.save((s.cpu(), r.cpu(), fs.cpu(), fr.cpu()), result)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,nq,dtype", [(2, 40_000, 256, "bf16"), (2, 9_999, 3, "f32"), (3, 20_000, 100, "f16")])
def test_sharded_gpu_search_equals_whole(world, n, nq, dtype, tmp_path):
    out = str(tmp_path / "rank0.pt")
    mp.start_processes(_worker, args=(world, _free_port(), n, nq, 10, dtype, out), nprocs=world, start_method="spawn")
    s, r, fs, fr = torch.load(out, weights_only=True)
    # one score rule for every plan (fl32 of the f64 dot, score desc / row asc): the sharded answer is the
    # whole index's bit for bit
    assert torch.equal(r, fr)
    assert torch.equal(s, fs)


def _ivf_worker(rank, world, port, n, nq, result):
    import torch.distributed as dist

    from rfx import dist as rdist
    from rfx.ivf import IvfIndex, synth_clustered

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dim, nlist = 256, 32
    r0, r1 = rdist.shard_range(n, rank, world)
    sh = rdist.ShardedIvf(IvfIndex(dim, nlist), r0)
    sample = synth_clustered(7, 48, 5, 0, 2048, dim, "bf16") if rank == 0 else None
    sh.train(sample, iters=3)
    sh.ivf.add(synth_clustered(7, 48, 5, r0, r1 - r0, dim, "bf16"))
    q = synth_clustered(7, 48, 99, 0, nq, dim, "bf16")
    s, r = sh.search(q, 10, 6)
    if rank == 0:
        full = IvfIndex(dim, nlist)
        full.train(sample, iters=3)
        full.add(synth_clustered(7, 48, 5, 0, n, dim, "bf16"))
        fs, fr = full.search(q, 10, 6)
        torch.save((s.cpu(), r.cpu(), fs.cpu(), fr.cpu()), result)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ivf_equals_whole(world, tmp_path):
    # one quantiser trained on rank 0 and broadcast; each rank its rows' part of every list
    out = str(tmp_path / "rank0.pt")
    mp.start_processes(_ivf_worker, args=(world, _free_port(), 9000, 64, out), nprocs=world, start_method="spawn")
    s, r, fs, fr = torch.load(out, weights_only=True)
    assert torch.equal(r, fr) and torch.equal(s, fs)
