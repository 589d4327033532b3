"""Benchmark: top-k retrieval QPS + achieved HBM GB/s (BASELINE.json metric).

Workload (BASELINE.json configs[2], the config the metric is quoted on):
  10M × 768 bf16 corpus (synthetic, counter-based generator, rows L2-normalised), batches of 256
  queries (bf16), brute-force top-10.  With --gpus N the corpus is row-sharded over N ranks
  (one process per GPU) and each step ends with the all-gather of per-shard top-k + merge
  (rfx.dist) — total work fixed => "scaling": "strong".
A step = one batch: fused MFMA scan + per-shard merge (+ all-gather + global merge for N > 1),
inputs already resident in HBM.  For N > 1 the shard's top-k goes out as packed records
(rfx_topk_merge_records), one RCCL all-gather issued from inside librfx (rfx_allgather_records on
an rfx_comm_init_rank communicator), one HIP merge of the gathered records.  torch.distributed
(gloo) is only the control plane: the RCCL id bootstrap, barriers and the max-over-ranks timing.

The scan (--scan): "auto" (default) runs the exact two-pass scan wherever it applies (bf16/f16,
d 768/1024, 64 < nq, k <= 10: int8 screen kernel 10 over an int8 copy of the store built at load
time, exact bf16 re-score of the survivors, the exact kernel 6/8 as a device-gated fallback;
DESIGN §4.10); "exact" runs the one-pass exact scan (kernel 6 at config 3).  Both return the
oracle's top-k; the roofline is priced on the bytes the timed kernel actually reads.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--nq Q] [--k K] [--dim D]
                       [--dtype bf16|f16|f32] [--scan auto|exact] [--no-cpu-baseline]
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "top-k retrieval QPS + achieved HBM GB/s, 10M×768 k=10, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec; 6.29 TB/s measured float4 copy)
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 matrix (v_mfma_f32_16x16x4_f32)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16/f16 MFMA (no sparsity)
I8_MFMA_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: i8 MFMA = 2x the bf16 rate (dense)
HBM_COPY_GBPS = 6290.0  # MI355X_MICROARCH.md: measured float4 copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample-rows", type=int, default=1_000_000)
    # corpus copies the steps rotate through: a corpus smaller than the 256 MB Infinity Cache
    # would otherwise be re-read from the cache (config 2: 307 MB); 0 = enough copies that
    # ~768 MB of other rows pass between two reads of one copy
    ap.add_argument("--copies", type=int, default=0)
    ap.add_argument("--scan", default="auto", choices=["auto", "exact"],
                    help="auto: the exact two-pass scan (int8 screen + exact re-score) where it applies")
    ap.add_argument("--allow-host-exchange", action="store_true",
                    help="N > 1: if RCCL cannot be initialised, exchange through host memory instead of failing")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # oracle check of the last timed step (rank 0; at N > 1 the gathered answer): every `stride`-th
    # query against oracle.search.topk_blocks over ALL rows (after the timed region); 0 = off
    ap.add_argument("--oracle-stride", type=int, default=4)
    # An event record is not free on this GPU (~5 us each, measured: profiles/r04k/): the N > 1 step
    # records 5 per instrumented step, 26 us of a 0.38-ms shard step.  0 = auto: instrument 4 of the
    # timed steps (every steps/4-th), so the line's ms_per_step carries ~1/5 of that cost
    ap.add_argument("--event-stride", type=int, default=0,
                    help="bracket every Nth timed step with HIP events (kernel_ms = their average); 0 = steps // 4")
    # rehearsal of the multi-GPU path on a one-GPU box: gloo transport, every rank on cuda:0,
    # and --check compares the sharded result with a whole-index search on rank 0
    ap.add_argument("--backend", default="rccl", choices=["rccl", "gloo"])
    ap.add_argument("--one-device", action="store_true")
    ap.add_argument("--check", action="store_true")
    # the N > 1 step (records, RCCL all-gather, gathered merge, per-phase timings) at world 1:
    # a 1-rank RCCL communicator from librfx (rfx_comm_init_rank), so the path runs on a 1-GPU box
    ap.add_argument("--force-comm", action="store_true")
    # RCCL exchange of the N > 1 step: "gather" (default) = every rank's records to rank 0, where the
    # answer is assembled (grouped send / recv, one hop); "allgather" = every rank gets all records
    ap.add_argument("--exchange", default="gather", choices=["gather", "allgather"])
    # the N > 1 step over RCCL with the two-pass plan: batch i's select, fallback, exchange and gathered
    # merge run on stream B (CU 0 of every XCD) while batch i + 1's screen runs on stream A (the other
    # CUs, kernel 10 on 248 workgroups); double-buffered workspaces.  Off by default: measured slower
    # (profiles/r04n/: 0.60 against 0.377 ms per shard step — the screen on the masked CUs and the select
    # on 8 CUs both lose more than the overlap hides)
    ap.add_argument("--pipeline", default="off", choices=["on", "off"])
    ap.add_argument("--reserve-cus", type=int, default=8,
                    help="--pipeline: CUs (bits 0..n-1 of the CU mask) for stream B; 0 = two unmasked streams")
    return ap.parse_args()


def workload_name(a):
    """BASELINE.json config this shape is (configs[1..3]); anything else is a custom shape."""
    shape = (a.rows, a.dim, a.dtype, a.nq, a.k)
    if shape == (10_000_000, 768, "bf16", 256, 10):
        return "cfg3"
    if shape == (100_000, 768, "f32", 1, 10):
        return "cfg2"
    if shape[1:] == (1024, "f16", 256, 10) and a.rows in (12_500_000, 100_000_000):
        return "cfg4" + (" (one GPU's shard)" if a.rows == 12_500_000 else "")
    return "custom"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


KERNEL_NAMES = {0: "scan_valu_kernel", 1: "scan_mfma_kernel", 2: "scan_mfma2_kernel", 3: "scan_mfma3_kernel",
                4: "scan_mfma4_kernel", 5: "scan_mfma5_kernel", 6: "scan_mfma6_kernel",
                7: "scan_mfma7_kernel", 8: "scan_mfma8_kernel", 9: "scan_mfma9_kernel", 10: "scan_screen_kernel",
                11: "screen_valu_kernel"}
SCAN_NAMES = {0: "valu", 1: "mfma128", 2: "mfma256", 3: "mfma_qstationary128", 4: "mfma_qstationary256",
              5: "mfma_qstationary256_2wps", 6: "mfma16_qstationary256_2wps", 7: "mfma16_qstationary128_2wps_xcdpair",
              8: "mfma16_qstationary128_ksplit_pairs_xcdpair", 9: "mfma_f32_qstationary128",
              10: "two_pass: i8 mfma16x16x64 screen (qstationary256_2wps) + exact re-score + gated exact fallback",
              11: "two_pass_valu: i8 dot4 screen + exact re-score + merge in one launch, gated exact one-launch fallback"}


def load_pmc_traffic(workload_key, kernel_name):
    """HBM bytes per scan launch from the committed rocprofv3 PMC summary (profiles/), or None —
    also None when that summary was taken on another kernel than the one this run launched."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        e = d.get(workload_key)
        if e is None or e.get("kernel_match") not in kernel_name:
            return None
        return float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.one_device:
        local = 0
        a.backend = "gloo"  # RCCL refuses two ranks on one GPU: the rehearsal exchanges via the host
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")  # control plane only (bootstrap, barriers, timing)

    from rfx import dist as rdist
    from rfx._lib import RfxCapacityError
    from rfx.index import DeviceIndex, synth_rows

    comm, exchange_note = None, None
    multi = world > 1 or a.force_comm  # the sharded step: records -> all-gather -> gathered merge
    if world == 1 and a.force_comm:
        comm = rdist.RcclComm.for_rank(1, 0, local, rdist.RcclComm.unique_id())
    if world > 1 and a.backend == "rccl":
        # every rank must take the same exchange: agree on RCCL's init over the gloo control plane.
        # A failed init ends the run unless --allow-host-exchange (then the JSON line says so)
        ok, err = 1, ""
        try:
            comm = rdist.RcclComm.from_process_group(local)
        except Exception as e:  # noqa: BLE001 (any init failure: reported below)
            ok, err = 0, f"{type(e).__name__}: {e}"
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag[0]):
            if comm is not None:
                comm.close()
            comm = None
            exchange_note = f"RCCL communicator init failed on some rank ({err or 'see that rank'}); host (gloo) exchange"
            print(exchange_note, file=sys.stderr, flush=True)
            if not a.allow_host_exchange:
                dist.destroy_process_group()
                raise SystemExit("RCCL init failed and --allow-host-exchange was not given: no host-exchange number")

    dev = torch.device("cuda", local)
    r0, r1 = rdist.shard_range(a.rows, rank, world)
    n_local = r1 - r0
    esz = {"bf16": 2, "f16": 2, "f32": 4}[a.dtype]
    # the exact two-pass scan: kernel 10 for batches (nq > 8, k <= 10: the 2-wave kernel up to 64 questions, the
    # 8-wave one above; bf16 / f16 at d 768 / 1024, f32 at d 768), kernel 11 for a few questions (any dtype,
    # nq <= 8, 5 <= k <= 16; config 2)
    screen = a.scan == "auto" and a.dim in (768, 1024) and (
        (a.nq > 8 and a.k <= 10 and (a.dtype in ("bf16", "f16") or a.dim == 768)) or (a.nq <= 8 and 5 <= a.k <= 16))
    row_bytes = a.dim if screen else a.dim * esz  # what a scan streams per row
    copies = a.copies or min(8, max(1, -(-(768 << 20) // max(n_local * row_bytes, 1)) + 1))
    if copies > 1 and n_local * row_bytes > (1 << 30):
        copies = 1  # far beyond the Infinity Cache already
    ixs, build_s, scan_note = [], 0.0, None
    for _ in range(copies):
        c = DeviceIndex(a.dim, a.dtype, local, capacity=n_local)
        c.add_synthetic(a.seed, n_local, gen_row0=r0)
        ixs.append(c)
        if screen:  # the int8 copy is part of the index (built at load / ingest time, not per batch)
            torch.cuda.synchronize()
            tb = time.perf_counter()
            try:
                c.enable_screen(1)
            except RfxCapacityError as e:
                # the copy does not fit beside the rows (config 4 whole on one GPU: 204.8 GB f16 + 102.4 GB
                # codes > 288 GB): the exact scan for every copy, said in the JSON line
                for x in ixs:
                    x.enable_screen(0)
                screen = False
                scan_note = f"--scan auto: int8 copy does not fit ({e}); exact scan"
                print(scan_note, file=sys.stderr, flush=True)
            build_s += time.perf_counter() - tb
    ix = ixs[0]
    q = synth_rows(a.seed + 1, 0, a.nq, a.dim, a.dtype, local)
    kern = ix.search_plan(a.nq, a.k)
    kname = KERNEL_NAMES[kern]
    rec = torch.empty((a.nq, a.k, 2), dtype=torch.int64, device=dev)
    ws = torch.empty(max(ix.workspace_bytes(a.nq, a.k), 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    gathered = torch.empty((world, a.nq, a.k, 2), dtype=torch.int64, device=dev) if multi else None
    torch.cuda.synchronize()

    from rfx import _lib
    from rfx._lib import check, lib, ptr, stream_ptr

    out_s = torch.empty((a.nq, a.k), dtype=torch.float32, device=dev)
    out_r = torch.empty((a.nq, a.k), dtype=torch.int64, device=dev)
    mg_s = torch.empty((a.nq, a.k), dtype=torch.float32, device=dev)  # the gathered merge's answer (N > 1)
    mg_r = torch.empty((a.nq, a.k), dtype=torch.int64, device=dev)
    NEV = 5  # scan begin, scan end, search done (records / result), all-gather done, gathered merge done

    def new_events():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(NEV)]
        for x in e:  # materialise the hipEvent_t handles (created lazily on first record)
            x.record(stream)
        return e

    # ---- the pipelined N > 1 step (see --pipeline) ------------------------------------------------------
    pipe = multi and comm is not None and kern == 10 and a.pipeline == "on"
    pipe_cfg = None
    if pipe:
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        res = max(1, min(a.reserve_cus, ncu - 1))
        nw = -(-ncu // 32)
        # CU mask bit i = CU i; the driver deals a multi-XCD part's mask bits out to the XCDs in turn, so
        # bits 0 .. 7 are one CU of each of the 8 XCDs (checked on the box: kernel 10 on the other 248 CUs
        # runs at 256/248 of its full-chip time, profiles/r04*/)
        ma = (ctypes.c_uint32 * nw)(*[0xffffffff] * nw)
        mb = (ctypes.c_uint32 * nw)(*[0] * nw)
        for b in range(res):
            ma[b // 32] &= ~(1 << (b % 32)) & 0xffffffff
            mb[b // 32] |= 1 << (b % 32)
        if a.reserve_cus > 0:
            pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
            check(lib.rfx_stream_create_cu_mask(local, ma, nw, ctypes.byref(pa)))
            check(lib.rfx_stream_create_cu_mask(local, mb, nw, ctypes.byref(pb)))
            sA = torch.cuda.ExternalStream(pa.value, device=dev)
            sB = torch.cuda.ExternalStream(pb.value, device=dev)
            scan_blocks = ncu - res
        else:  # --reserve-cus 0: two plain streams over the whole chip; the hardware fills CUs that batch i's
            # small kernels free with batch i+1's screen workgroups (no mask, the full 256-block screen)
            res = 0
            sA, sB = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
            scan_blocks = 0
        wsP = [ws, torch.empty_like(ws)]
        recP = [rec, torch.empty_like(rec)]
        gathP = [gathered, torch.empty_like(gathered)]
        mgP = [(mg_s, mg_r), (torch.empty_like(mg_s), torch.empty_like(mg_r))]
        evK = [torch.cuda.Event(), torch.cuda.Event()]
        evD = [torch.cuda.Event(), torch.cuda.Event()]
        pipe_cfg = {"streams": 2, "scan_cus": ncu - res, "post_cus": res, "scan_blocks": scan_blocks,
                    "note": "batch i's select + gated fallback + exchange + gathered merge (stream B) overlap batch "
                            "i+1's quantiser + kernel 10 (stream A); double-buffered workspaces"}

    def pstep(i, ev=None):
        sl = i % 2
        h = ixs[i % copies].handle
        if i >= 2:
            sA.wait_event(evD[sl])  # batch i - 2 done with workspace / records slot sl
        if ev is not None:
            ev[0].record(sA)
        check(lib.rfx_search_staged(h, ptr(q), a.nq, a.k, None, 0, r0, None, None, ptr(recP[sl]), ptr(wsP[sl]),
                                    wsP[sl].numel(), 1, scan_blocks, ctypes.c_void_p(sA.cuda_stream)))
        if ev is not None:
            ev[1].record(sA)
        evK[sl].record(sA)
        sB.wait_event(evK[sl])
        check(lib.rfx_search_staged(h, ptr(q), a.nq, a.k, None, 0, r0, None, None, ptr(recP[sl]), ptr(wsP[sl]),
                                    wsP[sl].numel(), 2, scan_blocks, ctypes.c_void_p(sB.cuda_stream)))
        if ev is not None:
            ev[2].record(sB)
        if a.exchange == "gather":
            comm.gather_records([recP[sl]], [gathP[sl] if rank == 0 else None], [sB], root=0)
        else:
            comm.allgather_records([recP[sl]], [gathP[sl]], [sB])
        if ev is not None:
            ev[3].record(sB)
        res_ = None
        if a.exchange != "gather" or rank == 0:
            ms_, mr_ = mgP[sl]
            check(lib.rfx_merge_gathered(ptr(gathP[sl]), world, a.nq, a.k, ptr(ms_), ptr(mr_),
                                         ctypes.c_void_p(sB.cuda_stream)))
            res_ = (ms_, mr_)
        if ev is not None:
            ev[4].record(sB)
        evD[sl].record(sB)
        return res_

    def step(i, ev=None):
        if pipe:
            return pstep(i, ev)
        h = ixs[i % copies].handle
        e0 = ctypes.c_void_p(ev[0].cuda_event) if ev is not None else None
        e1 = ctypes.c_void_p(ev[1].cuda_event) if ev is not None else None
        if not multi:
            check(lib.rfx_search_timed(h, ptr(q), a.nq, a.k, None, 0, 0, ptr(out_s), ptr(out_r), None, ptr(ws),
                                       ws.numel(), stream_ptr(stream), e0, e1))
            if ev is not None:
                ev[2].record(stream)
            return out_s, out_r
        # rank-local top-k as all-gather records (global rows), one collective, one HIP merge
        check(lib.rfx_search_timed(h, ptr(q), a.nq, a.k, None, 0, r0, None, None, ptr(rec), ptr(ws), ws.numel(),
                                   stream_ptr(stream), e0, e1))
        if ev is not None:
            ev[2].record(stream)
        if comm is not None:
            if a.exchange == "gather":
                comm.gather_records([rec], [gathered if rank == 0 else None], [stream], root=0)
                if rank != 0:  # the answer is rank 0's: nothing to merge here
                    if ev is not None:
                        ev[3].record(stream)
                        ev[4].record(stream)
                    return None
            else:
                comm.allgather_records([rec], [gathered], [stream])
            g = gathered
        else:  # --one-device rehearsal / --allow-host-exchange: through host memory (gloo)
            with torch.cuda.stream(stream):
                host = rec.cpu()
                parts = [torch.empty_like(host) for _ in range(world)]
                dist.all_gather(parts, host)
                g = torch.stack(parts).to(dev)
        if ev is not None:
            ev[3].record(stream)
        check(lib.rfx_merge_gathered(ptr(g), world, a.nq, a.k, ptr(mg_s), ptr(mg_r), stream_ptr(stream)))
        if ev is not None:
            ev[4].record(stream)
        return mg_s, mg_r

    for i in range(a.warmup):
        step(i)
    stride = a.event_stride if a.event_stride > 0 else max(1, a.steps // 4)
    ev_steps = list(range(0, a.steps, stride))
    evs = {i: new_events() for i in ev_steps}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        out = step(i, evs.get(i))
    host_issue = time.perf_counter() - t0  # host time to enqueue the K steps (GPU-bound when < elapsed)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    def avg(i, j):
        return sum(e[i].elapsed_time(e[j]) for e in evs.values()) / len(evs)

    scan_ms = avg(0, 1)
    phases = {"scan_ms": scan_ms, "search_done_ms": avg(0, 2)}
    if multi:
        phases.update({"records_merge_ms": avg(1, 2), "exchange_ms": avg(2, 3), "gathered_merge_ms": avg(3, 4)})
    if world > 1:
        t = torch.tensor([elapsed] + list(phases.values()), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        phases = {k_: float(v) for k_, v in zip(phases, t[1:].tolist())}
        scan_ms = phases["scan_ms"]
    if a.check:  # the global top-k of the last step equals one whole-index search (exact)
        if rank == 0:
            got_s, got_r = out
            full = DeviceIndex(a.dim, a.dtype, local, capacity=a.rows)
            full.add_synthetic(a.seed, a.rows)
            if screen:  # the same scan as the shards (its scores are the exact re-score's)
                full.enable_screen(1)
            ref_s, ref_r = full.search(q, a.k)
            if not (torch.equal(got_r, ref_r) and torch.equal(got_s, ref_s)):
                raise SystemExit("--check: sharded result differs from the whole-index search")
            print("check ok: sharded top-k == whole-index top-k", flush=True)
            del full

    # algorithmic bytes of one scan launch on the largest shard: rows read once,
    # queries read once, (score,row) results written once.  The two-pass scan's kernel 10 reads the
    # int8 codes (dim B per row), the 16-B record {scale, live word} of every 32-row tile, the int8
    # query codes and their bounds, and writes its candidate lists (KL (score, row) pairs per query
    # and list) and one drop word per (query, list): its roofline is priced on THOSE bytes, not on
    # the bf16 rows it does not read.
    n_max = rdist.shard_range(a.rows, 0, world)[1]
    nq_pad = -(-a.nq // 256) * 256
    if kern == 10:
        ntiles = -(-n_max // 32)
        if a.nq <= 64:  # the 2-wave kernel (k_screen.hip plan_scan_screen): 64 queries, up to 512 workgroups
            nq_pad = 64
            blocks = min(int(os.environ.get("RFX_SCREEN_W2_BLOCKS", "0")) or 512, max(ntiles // 12, 8))
            blocks = max(min(blocks // 8 * 8 if blocks > 8 else blocks, ntiles), 1)
        else:
            blocks = min(256 // max(1, nq_pad // 256), ntiles)
        # lists per (query, workgroup): 2 (32 queries per wave), 1 with the 64-queries-per-wave kernel (RFX_K10_Q64)
        n_lists = (1 if (a.nq > 64 and a.dim == 768 and os.environ.get("RFX_K10_Q64") == "1") else 2) * blocks
        kl = 4 if a.k <= 4 else 10
        alg_bytes = (n_max * a.dim + (-(-n_max // 32)) * 16 + nq_pad * a.dim + nq_pad * 4
                     + a.nq * n_lists * (kl * 8 + 4))
    elif kern == 11:
        # int8 codes + tile records + the raw queries + the per-block candidate lists (16 x (f32, i32))
        # written and read back by the last block + the results (re-scored rows: a few per query)
        rpw = -(-max(16, -(-n_max // 1024)) // 4) * 4  # plan_scan_valu: rows per wave, 4 waves per block
        n_lists = -(-(-(-n_max // rpw)) // 4)
        alg_bytes = (n_max * a.dim + (-(-n_max // 32)) * 16 + a.nq * a.dim * esz + 2 * a.nq * n_lists * 16 * 8
                     + a.nq * a.k * 12)
    else:
        alg_bytes = n_max * a.dim * esz + a.nq * a.dim * esz + a.nq * a.k * 12
    achieved = alg_bytes / (scan_ms * 1e-3) / 1e9
    qps = a.nq * a.steps / elapsed
    workload_key = f"{a.rows}x{a.dim}-{a.dtype}-nq{a.nq}-k{a.k}-g{world}" + ("-screen" if kern in (10, 11) else "")
    result = {
        "metric": METRIC,
        "value": round(qps, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (splitmix64 counter-based corpus + queries, rows L2-normalised; oracle/synth.py)",
        "config": {"workload": f"{workload_name(a)}: {a.rows}x{a.dim} {a.dtype} corpus row-sharded over {world} "
                               f"GPU(s), {a.nq} queries/batch, brute-force top-{a.k}",
                   "rows": a.rows, "dim": a.dim, "nq": a.nq, "k": a.k, "parallelism": f"rowshard{world}",
                   "corpus_copies": copies, "scan": a.scan,
                   "exchange": (("RCCL gather to rank 0 from librfx (rfx_gather_records: grouped send/recv)"
                                 if a.exchange == "gather" else "RCCL all-gather from librfx (rfx_allgather_records)")
                                if comm is not None else
                                exchange_note if exchange_note else
                                "host (gloo) rehearsal" if world > 1 else "none (one shard)"),
                   "scan_kernel": SCAN_NAMES[kern] + (f" ({scan_note})" if scan_note else ""),
                   "pipeline": pipe_cfg},
        "achieved_hbm_gbps_per_gpu": round(achieved, 1),
        "build_id": _lib.BUILD_ID,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": load_pmc_traffic(workload_key, kname),
                     "kernel": kname,
                     "kernel_ms": round(scan_ms, 4), "event_timed_launches": len(evs), "event_stride": stride,
                     "alg_bytes_per_launch": alg_bytes},
        "phases_ms": {k_: round(v, 4) for k_, v in phases.items()},
        "host_issue_ms_per_step": round(host_issue / a.steps * 1e3, 4),
    }
    if comm is not None:
        result["config"]["rccl"] = {"world": comm.world, "rank_of_reporter": comm.rank, "n_local": comm.n_local}
    # MFMA utilisation alongside the HBM roofline (bf16/f16 dense peak), and the fraction
    # of the measured copy bandwidth (MI355X_MICROARCH.md: 6.29 TB/s float4 copy)
    flops = 2.0 * n_max * a.dim * a.nq
    if kern in (1, 2, 3, 6, 7, 8):
        result["roofline"]["mfma_tflops"] = round(flops / (scan_ms * 1e-3) / 1e12, 1)
        result["roofline"]["mfma_frac_of_dense_peak"] = round(flops / (scan_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4)
    if kern == 10:  # int8 ops on the padded query group
        tops = 2.0 * n_max * a.dim * nq_pad / (scan_ms * 1e-3) / 1e12
        result["roofline"]["mfma_i8_tops"] = round(tops, 1)
        result["roofline"]["mfma_frac_of_i8_dense_peak"] = round(tops / I8_MFMA_PEAK_TOPS, 4)
    result["roofline"]["frac_of_measured_copy_bw"] = round(achieved / HBM_COPY_GBPS, 4)
    if kern == 9:  # f32 MFMA is 1/16 of the bf16 rate: this scan is matrix-core bound, not HBM bound
        tflops = flops / (scan_ms * 1e-3) / 1e12
        result["roofline"].update({"bound": "mfma", "achieved": round(tflops, 2), "peak": F32_MFMA_PEAK_TFLOPS,
                                   "unit": "TFLOP/s", "frac": round(tflops / F32_MFMA_PEAK_TFLOPS, 4),
                                   "hbm_gbps": round(achieved, 1)})
    if kern == 10:
        # the whole two-pass step's reads: kernel 10's bytes + the select kernel's (candidate lists,
        # the bf16 queries, the survivors' bf16 rows) — what one batch costs in HBM traffic
        diag, fb = ixs[(a.steps - 1) % copies].screen_diag(a.nq, a.k, ws)
        sv = diag[:, 1]
        sel_bytes = int(a.nq * n_lists * (kl * 8 + 4) + a.nq * a.dim * esz + max(int(sv.sum()), 0) * a.dim * esz)
        step_bytes = alg_bytes + sel_bytes
        result["two_pass"] = {
            "int8_copy_build_s": round(build_s / copies, 3), "int8_copy_bytes": n_max * a.dim,
            "kept_mean": round(float(diag[:, 0].mean()), 1), "survivors_mean": round(float(sv.mean()), 1),
            "survivors_max": int(sv.max()), "fallback_ran": bool(fb),
            "step_bytes": step_bytes, "step_gbps": round(step_bytes / (elapsed / a.steps) / 1e9, 1),
            "step_frac_of_hbm_peak": round(step_bytes / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBPS, 4),
            "note": "step_bytes = kernel 10's bytes + select (candidate lists, bf16 queries, survivor rows)"}

    check_ok = True
    if rank == 0 and a.oracle_stride > 0 and out is not None:
        if multi:
            # rank 0 holds the gathered answer (global rows) but only its own shard: the oracle reads
            # every shard's rows from the same counter-based generator the ranks built them from
            def read(r, n):
                return synth_rows(a.seed, r, n, a.dim, a.dtype, local)
        else:
            read = ix.read
        result["oracle_check"] = oracle_check(read, a.rows, q, out, a)
        result["oracle_check"]["answer"] = "gathered merge (rank 0)" if multi else "single shard"
        check_ok = result["oracle_check"]["ok"]
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(ix, q, a)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not check_ok:
        raise SystemExit("oracle check of the last timed step FAILED (see oracle_check in the JSON line)")


def oracle_check(read, n_rows, q, out, a):
    """Checker (not timed): the last timed step's top-k for every a.oracle_stride-th query against
    the CPU oracle over ALL rows of the corpus, read 1M rows at a time (`read(row0, n)`: back from
    HBM at N = 1; regenerated on rank 0 for the gathered answer of N > 1) and widened exactly to f32
    on the host (oracle.search.topk_blocks: f32 screen with a rigorous rounding bound + exact
    rescoring).  Parity rule: oracle.search.check_topk (1e-5 / 2e-6)."""
    import numpy as np

    from oracle import search as osearch

    t0 = time.perf_counter()
    sel = list(range(0, a.nq, a.oracle_stride))
    q64 = q[sel].cpu().float().numpy().astype(np.float64)
    blk = 1 << 20

    def blocks():
        for r0 in range(0, n_rows, blk):
            yield r0, read(r0, min(blk, n_rows - r0)).cpu().float().numpy()

    ref_s, ref_r = osearch.topk_blocks(q64, blocks(), a.k)
    got_s, got_r = out[0][sel].cpu().numpy(), out[1][sel].cpu().numpy()

    def scores_of(qi, rows):
        return np.array([read(int(x), 1).cpu().float().numpy()[0].astype(np.float64) @ q64[qi] for x in rows])

    probs = osearch.check_topk(got_s, got_r, ref_s, ref_r, scores_of, tol=1e-5, tie_band=2e-6)
    same = got_r == ref_r
    err = float(np.abs(got_s[same].astype(np.float64) - ref_s[same]).max()) if same.any() else 0.0
    return {"ok": not probs, "queries": len(sel), "rows": n_rows, "problems": probs[:3],
            "rows_identical_frac": round(float(same.mean()), 6), "max_abs_score_err": err,
            "rule": "oracle.search.check_topk tol 1e-5, tie band 2e-6", "secs": round(time.perf_counter() - t0, 1)}


def cpu_baseline(ix, q, a):
    """Oracle (numpy) top-k on the host cores over a bounded row sample, extrapolated to the
    full corpus (QPS = nq / (t_sample * rows / sample_rows))."""
    import numpy as np

    from oracle import baseline, synth

    n = min(a.cpu_sample_rows, ix.rows)
    stored = ix.read(0, n).cpu()
    if a.dtype == "bf16":
        stored = stored.view(torch.int16).numpy().view(np.uint16)
    else:
        stored = stored.numpy()
    qh = q.cpu()
    q64 = synth.to_f64(qh.view(torch.int16).numpy().view(np.uint16) if a.dtype == "bf16" else qh.numpy(), a.dtype)
    secs, _, _ = baseline.time_topk(stored, a.dtype, q64, a.k)
    full = secs * a.rows / n
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    out = {"value": round(a.nq / full, 2), "unit": "queries/s", "cores": threads, "kind": "port",
           "sample": f"oracle numpy top-{a.k} of {a.nq} queries over rows 0..{n} of the same corpus "
                     f"({secs:.2f} s), extrapolated x{a.rows / n:.1f} to {a.rows} rows",
           "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "mock_restatement_us_per_call": round(baseline.time_mock_plumbing(), 2)}
    # the same sample at every host CPU the box shows (OMP_NUM_THREADS is the box's
    # share, os.cpu_count() the whole machine's)
    allc = os.cpu_count() or threads
    if allc != threads:
        try:
            from threadpoolctl import threadpool_limits
            with threadpool_limits(limits=allc):
                secs2, _, _ = baseline.time_topk(stored, a.dtype, q64, a.k)
            out["at_os_cpu_count"] = {"value": round(a.nq / (secs2 * a.rows / n), 2), "cores": allc}
        except Exception as e:  # noqa: BLE001 (reported, not fatal)
            out["at_os_cpu_count"] = {"error": f"{type(e).__name__}: {e}"}
    return out


if __name__ == "__main__":
    main()
