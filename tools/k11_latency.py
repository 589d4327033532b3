"""Kernel 11's latency under concurrency (DESIGN §4.10b "Round 6").

A lone question's search (config 2: 100k x 768 f32, k 10, kernel 11) is timed from the host as a chat
thread sees it: issue, then wait for its stream.  Scenarios, each over a fixed count of searches:
  solo        kernel 11 alone on the device;
  beside_k10  a second thread keeps kernel-10 batches (2M x 768 bf16, nq 256, a workgroup per CU at
              launch_bounds(512, 1)) queued on another stream the whole time;
  two_k11     two threads, each with its own config-2 store and stream, search at once (kernel-11
              launches of one device are ordered by librfx once two streams issue them; run with
              RFX_K11_UNORDERED=1 to see them overlap).
Every answer of the timed searches is checked against the same search run alone first (bit-identical).
Prints one JSON object: per scenario, latency percentiles in microseconds."""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

import rfx.index as ri  # noqa: E402


def pct(v):
    a = np.sort(np.asarray(v)) * 1e6
    return {"n": int(a.size), "p50": round(float(np.percentile(a, 50)), 1), "p90": round(float(np.percentile(a, 90)), 1),
            "p99": round(float(np.percentile(a, 99)), 1), "max": round(float(a[-1]), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--searches", type=int, default=2000)
    ap.add_argument("--k10-rows", type=int, default=2_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    k = 10
    ix_a = ri.DeviceIndex(768, "f32")
    ix_a.add_synthetic(61, 100_000)
    ix_a.enable_screen(1)
    ix_c = ri.DeviceIndex(768, "f32")
    ix_c.add_synthetic(62, 100_000)
    ix_c.enable_screen(1)
    ix_b = ri.DeviceIndex(768, "bf16")
    ix_b.add_synthetic(63, a.k10_rows)
    ix_b.enable_screen(1)
    assert ix_a.search_plan(1, k) == 11 and ix_c.search_plan(1, k) == 11 and ix_b.search_plan(256, k) == 10
    qa = ri.synth_rows(64, 0, a.searches, 768, "f32")
    qc = ri.synth_rows(65, 0, a.searches, 768, "f32")
    qb = ri.synth_rows(66, 0, 256, 768, "bf16")
    s_a, s_b, s_c = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    ws_a = torch.empty(ix_a.workspace_bytes(1, k), dtype=torch.uint8, device=dev)
    ws_c = torch.empty(ix_c.workspace_bytes(1, k), dtype=torch.uint8, device=dev)
    ws_b = torch.empty(ix_b.workspace_bytes(256, k), dtype=torch.uint8, device=dev)

    def one(ix, q, ws, st):
        with torch.cuda.stream(st):
            t0 = time.perf_counter()
            s, r = ix.search(q, k, workspace=ws, stream=st)
            st.synchronize()
            return time.perf_counter() - t0, s, r

    # answers alone, the check for every timed search
    ref_a = [one(ix_a, qa[i:i + 1], ws_a, s_a)[1:] for i in range(a.searches)]
    ref_c = [one(ix_c, qc[i:i + 1], ws_c, s_c)[1:] for i in range(a.searches)]
    for i in range(50):  # warm the kernel-10 path
        one(ix_b, qb, ws_b, s_b)

    def run(ix, q, ws, st, ref, lat, bad):
        for i in range(a.searches):
            dt, s, r = one(ix, q[i:i + 1], ws, st)
            lat.append(dt)
            if not (torch.equal(s, ref[i][0]) and torch.equal(r, ref[i][1])):
                bad.append(i)

    out = {"rows": 100_000, "dim": 768, "dtype": "f32", "k": k, "k10_rows": a.k10_rows,
           "unordered": os.environ.get("RFX_K11_UNORDERED", "0") == "1"}
    # solo
    lat, bad = [], []
    run(ix_a, qa, ws_a, s_a, ref_a, lat, bad)
    out["solo"] = pct(lat) | {"wrong": len(bad)}
    # kernel 11 beside a stream of kernel-10 batches
    stop = threading.Event()
    k10_n = [0]

    def feed():
        with torch.cuda.stream(s_b):
            while not stop.is_set():
                for _ in range(4):
                    ix_b.search(qb, k, workspace=ws_b, stream=s_b)
                k10_n[0] += 4
                s_b.synchronize()

    th = threading.Thread(target=feed)
    th.start()
    time.sleep(0.05)
    lat, bad = [], []
    t0 = time.perf_counter()
    run(ix_a, qa, ws_a, s_a, ref_a, lat, bad)
    wall = time.perf_counter() - t0
    stop.set()
    th.join()
    out["beside_k10"] = pct(lat) | {"wrong": len(bad), "k10_batches": k10_n[0], "wall_s": round(wall, 3)}
    # two kernel-11 streams at once
    lat_a, bad_a, lat_c, bad_c = [], [], [], []
    th = threading.Thread(target=run, args=(ix_c, qc, ws_c, s_c, ref_c, lat_c, bad_c))
    th.start()
    run(ix_a, qa, ws_a, s_a, ref_a, lat_a, bad_a)
    th.join()
    out["two_k11"] = {"a": pct(lat_a) | {"wrong": len(bad_a)}, "b": pct(lat_c) | {"wrong": len(bad_c)}}
    print(json.dumps(out))
    assert not (out["solo"]["wrong"] or out["beside_k10"]["wrong"] or bad_a or bad_c), "answers differ from solo"


if __name__ == "__main__":
    main()
