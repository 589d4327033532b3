"""GPU: the row-sharded store behind the drop-in adapter (rfx.sharded.ShardedIndex, RFX_DEVICES)
and the RCCL communicator inside the C ABI (rfx_comm_* / rfx_allgather_records).

On the one-GPU box the shards are logical (RFX_DEVICES=0x4: four row ranges on cuda:0; the
exchange is a device-local stack); the RCCL path is exercised by a 1-rank communicator in both
process models (ncclCommInitRank and ncclCommInitAll).  The 8-GPU run is the driver's."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DOCS = [("alpha beta gamma delta epsilon " * 40, {"tenant": "acme"}),
        ("zeta eta theta iota kappa lambda " * 35, {"tenant": "globex"}),
        ("mock mode document assistant retrieval citations " * 30, {"tenant": "acme"}),
        ("hbm bandwidth roofline matrix cores wavefront lds " * 33, None)]
QUESTIONS = ["alpha gamma", "theta kappa lambda", "document retrieval", "roofline lds", "beta zeta assistant"]


def _hits(ret, name, q, k, filt=None):
    return [(h.row, h.score, h.file_id) for h in ret.search([name], q, k, metadata_filter=filt)]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_sharded_adapter_equals_unsharded(tmp_path, dtype):
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever
    from rfx.sharded import ShardedIndex

    root = str(tmp_path)
    writer = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype=dtype)
    name = writer.create_store("shared")
    ids = [writer.add_document(name, t, f"doc{i}", {"white_space_config": {"max_tokens_per_chunk": 4}}, m)[0]
           for i, (t, m) in enumerate(DOCS)]
    plain = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype=dtype)
    sharded = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0, devices="0x4"), dtype=dtype)
    six = sharded.registry.get(name).index
    assert isinstance(six, ShardedIndex) and len(six.shards) == 4
    assert min(s.rows for s in six.shards) > 0 and six.rows == plain.registry.get(name).index.rows

    def same():
        for q in QUESTIONS:
            for k in (1, 5, 10):
                assert _hits(sharded, name, q, k) == _hits(plain, name, q, k)
            assert _hits(sharded, name, q, 7, {"tenant": "acme"}) == _hits(plain, name, q, 7, {"tenant": "acme"})

    same()
    # growth lands on the last shard; deletions anywhere
    before = [s.rows for s in six.shards]
    _, n_late = writer.add_document(name, "nu xi omicron pi rho sigma " * 20, "late", None, {"tenant": "acme"})
    writer.delete_file(name, ids[1])
    same()
    assert [s.rows for s in sharded.registry.get(name).index.shards] == before[:-1] + [before[-1] + n_late]

    # a batched search (MFMA kernels) straight on the indexes: bit-identical rows and scores
    pst = plain.registry.get(name)
    emb = plain.embedder(768)
    qs = emb.embed_texts([f"{w} {v}" for w in ("alpha", "theta", "roofline", "sigma") for v in range(64)], dtype)
    a_s, a_r = pst.index.search(qs, 10)
    b_s, b_r = six.search(qs, 10)
    assert torch.equal(a_r, b_r) and torch.equal(a_s, b_s)


def test_sharded_index_split_and_masks(tmp_path):
    """Shard bases are multiples of 32 (mask words never straddle shards); a masked batched
    search over 3 logical shards equals the unsharded masked search."""
    from rfx import filters
    from rfx.index import DeviceIndex
    from rfx.sharded import ShardedIndex

    n = 10_007
    whole = DeviceIndex(768, "bf16", 0)
    whole.add_synthetic(3, n)
    path = str(tmp_path / "rows.rfx")
    whole.rows_append(path, 0)
    sh = ShardedIndex(768, "bf16", [0, 0, 0])
    sh.rows_sync(path, n)
    assert all(b % 32 == 0 for b in sh.bases) and sh.rows == n
    words = filters.row_mask_words(n, [(5, 3000), (4100, 10), (9000, 1007)])
    q = whole.read(0, 300)[::3].contiguous()  # 100 queries
    m_whole = torch.from_numpy(words).cuda()
    a = whole.search(q, 10, row_mask=m_whole)
    b = sh.search(q, 10, row_mask=sh.mask_tensor(words))
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    sh.tombstone([6, 9000, 4105])
    whole.tombstone([6, 9000, 4105])
    a = whole.search(q[:5], 10)
    b = sh.search(q[:5], 10)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])


def _records(nq, k, seed):
    g = torch.Generator().manual_seed(seed)
    s = torch.rand((nq, k), generator=g).sort(dim=1, descending=True).values
    r = torch.randint(0, 1 << 40, (nq, k), generator=g)
    from rfx.dist import pack
    return pack(s, r).cuda()


def test_rccl_rank_communicator_one_rank():
    from rfx.dist import RcclComm, gather_merge_records

    comm = RcclComm.for_rank(1, 0, 0, RcclComm.unique_id())
    assert (comm.world, comm.rank, comm.n_local) == (1, 0, 1)
    rec = _records(256, 10, 1)
    out = torch.empty((1, 256, 10, 2), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    comm.allgather_records([rec], [out], [st])
    torch.cuda.synchronize()
    assert torch.equal(out[0], rec)
    s, r = gather_merge_records(rec, 10, comm=comm)
    assert torch.equal(r.cpu(), rec[..., 1].cpu())
    assert np.array_equal(s.cpu().numpy().view(np.int32), rec[..., 0].cpu().numpy().astype(np.int32))
    comm.close()


def test_rccl_group_communicator_one_device():
    from rfx.dist import RcclComm

    comm = RcclComm.for_devices([0])
    assert (comm.world, comm.n_local) == (1, 1)
    rec = _records(3, 5, 2)
    out = torch.zeros((1, 3, 5, 2), dtype=torch.int64, device="cuda")
    comm.allgather_records([rec], [out], [torch.cuda.current_stream()])
    torch.cuda.synchronize()
    assert torch.equal(out[0], rec)
    comm.close()


def test_sharded_resplit_device_to_device(tmp_path):
    """Growth past twice the mean re-splits device to device (no row-file reload): shard 0 keeps its
    rows, the others are rebuilt from peer copies; the result equals one index, tombstones kept."""
    from rfx.index import DeviceIndex
    from rfx.sharded import ShardedIndex

    whole = DeviceIndex(768, "bf16", 0)
    whole.add_synthetic(4, 9000)
    path = str(tmp_path / "rows.rfx")
    whole.rows_append(path, 0)
    sh = ShardedIndex(768, "bf16", [0, 0, 0])
    sh.rows_sync(path, 9000)
    gen0, first = sh.generation, sh.shards[0]
    sh.tombstone([17, 4000, 8999])
    whole.tombstone([17, 4000, 8999])
    whole.add_synthetic(4, 21000, gen_row0=9000)
    whole.rows_append(path, 9000)
    sh.rows_sync(path, 30000)  # last shard 3000 + 21000 rows > 2x the others' mean: re-split
    assert sh.generation > gen0 and sh.shards[0] is first
    assert all(b % 32 == 0 for b in sh.bases) and sh.rows == 30000
    assert max(s.rows for s in sh.shards) - min(s.rows for s in sh.shards) <= 64
    assert sh.live_rows == whole.live_rows
    q = whole.read(100, 200)[::2].contiguous()
    for nq in (100, 3):
        a = whole.search(q[:nq], 10)
        b = sh.search(q[:nq], 10)
        assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    assert torch.equal(sh.read(0, 30000).view(torch.int16), whole.read(0, 30000).view(torch.int16))


def test_sharded_ivf_store_equals_unsharded(tmp_path):
    """An RFX_INDEX=ivf store read through 4 logical shards (rfx.sharded.ShardedIvf: one list set
    per shard under the committed centroids, two record exchanges) answers bit-identically to the
    same store on one device, before and after growth that re-splits the shards."""
    from rfx import ivf as rivf
    from rfx import store as rstore
    from rfx.sharded import ShardedIndex, ShardedIvf

    dim, spec = 768, {"kind": "ivf", "nlist": 32, "nprobe": 8, "train_min": 4000}
    root = str(tmp_path)
    st = rstore.StoreRegistry(root=root, device=0).create("ivf-sh", dim, "bf16", spec=spec)
    docs = [rivf.synth_clustered(7, 48, 200 + i, 1500 * i, 1500, dim, "bf16") for i in range(3)]
    fids = [st.add_document([f"d{i}-{j}" for j in range(1500)], v, f"d{i}.md")[0] for i, v in enumerate(docs)]
    st.delete_file(fids[1])
    st.add_document([f"e-{j}" for j in range(3000)], rivf.synth_clustered(7, 48, 300, 0, 3000, dim, "bf16"), "e.md")
    assert st.ivf_ready()
    preg = rstore.StoreRegistry(root=root, device=0)
    sreg = rstore.StoreRegistry(root=root, device=0, devices="0x4")
    plain, shard = preg.get(st.name), sreg.get(st.name)
    assert isinstance(shard.index, ShardedIndex) and isinstance(shard.ivf, ShardedIvf)
    assert plain.ivf_ready() and shard.ivf_ready() and shard.ivf_id == plain.ivf_id
    q = rivf.synth_clustered(7, 48, 999, 0, 70, dim, "bf16")

    def same(k):
        a_s, a_r = plain.search(q, k)
        b_s, b_r = shard.search(q, k)
        assert np.array_equal(a_r.numpy(), b_r.numpy())
        assert np.array_equal(a_s.numpy().view(np.uint32), b_s.numpy().view(np.uint32))
        assert not np.isin(a_r.numpy(), np.arange(1500, 3000)).any()  # the deleted document

    for k in (1, 10, 20):
        same(k)
    # growth: the sharded reader's last shard passes twice the mean -> device-to-device re-split,
    # the lists are rebuilt on the new layout (26,000 live rows < 8x the trained 4,500: no retrain)
    gen = shard.index.generation
    st.add_document([f"g-{j}" for j in range(20000)], rivf.synth_clustered(7, 48, 400, 0, 20000, dim, "bf16"), "g.md")
    plain, shard = preg.get(st.name), sreg.get(st.name)
    assert shard.index.generation > gen and shard.ivf_id == plain.ivf_id
    assert shard.ivf_ready() and plain.ivf_ready()
    for k in (5, 10):
        same(k)


def test_rccl_gather_records_one_rank():
    """rfx_gather_records (grouped send/recv to the root) in both process models, world 1."""
    from rfx.dist import RcclComm

    rec = _records(256, 10, 3)
    st = torch.cuda.current_stream()
    comm = RcclComm.for_rank(1, 0, 0, RcclComm.unique_id())
    out = torch.zeros((1, 256, 10, 2), dtype=torch.int64, device="cuda")
    comm.gather_records([rec], [out], [st], root=0)
    torch.cuda.synchronize()
    assert torch.equal(out[0], rec)
    with pytest.raises(ValueError):
        comm.gather_records([rec], [None], [st], root=0)  # the root needs a receive buffer
    comm.close()
    comm = RcclComm.for_devices([0])
    out = torch.zeros((1, 256, 10, 2), dtype=torch.int64, device="cuda")
    comm.gather_records([rec], [out], [st], root=0)
    torch.cuda.synchronize()
    assert torch.equal(out[0], rec)
    comm.close()


def test_sharded_two_pass_equals_unsharded_screened(tmp_path):
    """every shard of a screened ShardedIndex searches with the exact two-pass scan
    (rfx_search_records: kernel 10 for the batch, kernel 11 + the records pack for a lone question), no
    shard falls back, and the answers are bit-identical to the unsharded screened index — unmasked,
    masked, and after tombstones."""
    from rfx import filters
    from rfx.index import DeviceIndex, synth_rows
    from rfx.sharded import ShardedIndex

    n = 200_003
    whole = DeviceIndex(768, "bf16", 0)
    whole.add_synthetic(21, n)
    path = str(tmp_path / "rows.rfx")
    whole.rows_append(path, 0)
    sh = ShardedIndex(768, "bf16", [0, 0, 0, 0])
    sh.rows_sync(path, n)
    whole.enable_screen(1)
    sh.enable_screen(1)
    q = synth_rows(22, 0, 256, 768, "bf16")
    for shard in sh.shards:
        assert shard.screen_state()[0] == 1
        assert shard.search_plan(256, 10) == 10 and shard.search_plan(1, 10) == 11
    a = whole.search(q, 10)
    b = sh.search(q, 10)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    for shard, base in zip(sh.shards, sh.bases):
        ws = torch.empty(shard.workspace_bytes(256, 10), dtype=torch.uint8, device="cuda")
        rec = shard.search_records(q, 10, row_offset=base, workspace=ws)
        diag, fb = shard.screen_diag(256, 10, ws)
        assert not fb and (diag[:, 1] >= 0).all()
        rows = rec[..., 1]
        assert ((rows >= base) & (rows < base + shard.rows)).all()
    for i in range(3):  # lone questions: kernel 11 on every shard, records through the pack launch
        a = whole.search(q[i:i + 1], 10)
        b = sh.search(q[i:i + 1], 10)
        assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    words = filters.row_mask_words(n, [(5, 30_000), (70_100, 10), (120_000, 50_007)])
    for nq in (256, 2):
        a = whole.search(q[:nq], 10, row_mask=torch.from_numpy(words).cuda())
        b = sh.search(q[:nq], 10, row_mask=sh.mask_tensor(words))
        assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    dead = np.unique(a[1][:, :3].cpu().numpy().ravel())
    whole.tombstone(dead)
    sh.tombstone(dead)
    for nq in (256, 1):
        a = whole.search(q[:nq], 10)
        b = sh.search(q[:nq], 10)
        assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
        assert not np.isin(b[1].cpu().numpy(), dead).any()


def test_sharded_screened_store_equals_unsharded(tmp_path, monkeypatch):
    """The adapter path: an RFX_DEVICES=0x4 store with RFX_SCREEN=1 answers bit-identically to the
    unsharded screened store, every shard on the two-pass plan."""
    from rfx import store as rstore
    from rfx.retriever import GpuRetriever

    monkeypatch.setenv("RFX_SCREEN", "1")
    root = str(tmp_path)
    writer = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
    name = writer.create_store("shared")
    for i, (t, m) in enumerate(DOCS):
        writer.add_document(name, t, f"doc{i}", {"white_space_config": {"max_tokens_per_chunk": 4}}, m)
    plain = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
    sharded = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0, devices="0x4"), dtype="bf16")
    six = sharded.registry.get(name).index
    assert all(s.screen_state()[0] == 1 and s.search_plan(256, 10) == 10 for s in six.shards)
    for qq in QUESTIONS:
        for k in (5, 10):
            assert _hits(sharded, name, qq, k) == _hits(plain, name, qq, k)
        assert _hits(sharded, name, qq, 7, {"tenant": "acme"}) == _hits(plain, name, qq, 7, {"tenant": "acme"})
    emb = plain.embedder(768)
    qs = emb.embed_texts([f"{w} {v}" for w in ("alpha", "theta", "roofline", "sigma") for v in range(64)], "bf16")
    a_s, a_r = plain.registry.get(name).index.search(qs, 10)
    b_s, b_r = six.search(qs, 10)
    assert torch.equal(a_r, b_r) and torch.equal(a_s, b_s)


@pytest.mark.parametrize("screen", [0, 1])
def test_sharded_search_one_c_call_equals_python_path(tmp_path, screen):
    """rfx_sharded_search (one C-ABI call: every shard's search, the exchange and the merge)
    returns the per-shard Python path's answer bit for bit — masked and unmasked, for batches of several
    sizes (its buffers are reused and grown), after growth that outgrows a shard's workspace, and against
    the unsharded index."""
    from rfx import filters
    from rfx.index import DeviceIndex
    from rfx.sharded import ShardedIndex

    n = 200_003
    whole = DeviceIndex(768, "bf16", 0)
    whole.add_synthetic(21, n)
    path = str(tmp_path / "rows.rfx")
    whole.rows_append(path, 0)
    sh = ShardedIndex(768, "bf16", [0, 0, 0, 0])
    sh.rows_sync(path, n)
    if screen:
        whole.enable_screen(1)
        sh.enable_screen(1)
    words = filters.row_mask_words(n, [(5, 30_000), (90_000, 70_000), (199_000, 1003)])
    m_whole = torch.from_numpy(words).cuda()
    for nq in (256, 3, 100, 256, 1):
        q = whole.read(7, nq * 5)[::5].contiguous()
        for mask in (None, words):
            sh.c_path = True
            c = sh.search(q, 10, row_mask=sh.mask_tensor(words) if mask is not None else None)
            sh.c_path = False
            p = sh.search(q, 10, row_mask=sh.mask_tensor(words) if mask is not None else None)
            w = whole.search(q, 10, row_mask=m_whole if mask is not None else None)
            assert torch.equal(c[0], p[0]) and torch.equal(c[1], p[1]), (nq, mask is not None)
            assert torch.equal(c[1], w[1]) and torch.equal(c[0], w[0]), (nq, mask is not None)
    # the last shard grows (its workspace must grow with it: the call regrows and retries once)
    whole.add_synthetic(21, 150_000, gen_row0=n)
    whole.rows_append(path, n)
    sh.rows_sync(path, n + 150_000)
    q = whole.read(11, 256 * 3)[::3].contiguous()
    sh.c_path = True
    c = sh.search(q, 10)
    w = whole.search(q, 10)
    assert torch.equal(c[1], w[1]) and torch.equal(c[0], w[0])
