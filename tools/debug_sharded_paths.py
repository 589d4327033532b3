"""Dev tool: a row-sharded index's search through the one-call C path and the per-shard Python path, each
on a fresh ShardedIndex, against the unsharded index, for small and large batches (and the per-shard
records of each path against each shard's own search_records on the default stream)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
import torch  # noqa: E402

from rfx.index import DeviceIndex  # noqa: E402
from rfx.sharded import ShardedIndex  # noqa: E402

n = 200_003
whole = DeviceIndex(768, "bf16", 0)
whole.add_synthetic(21, n)
path = "/tmp/dbg_rows.rfx"
whole.rows_append(path, 0)


def make():
    sh = ShardedIndex(768, "bf16", [0, 0, 0, 0])
    sh.rows_sync(path, n)
    return sh


for c_path in (False, True):
    sh = make()
    sh.c_path = c_path
    for nq in (3, 256, 3, 1, 8):
        q = whole.read(7, nq * 5)[::5].contiguous()
        w = whole.search(q, 10)
        got = sh.search(q, 10)
        torch.cuda.synchronize()
        ok = torch.equal(got[0], w[0]) and torch.equal(got[1], w[1])
        print({"c_path": c_path, "nq": nq, "equal_to_whole": ok}, flush=True)
        if not ok:
            for i, (s, b) in enumerate(zip(sh.shards, sh.bases)):
                rec = s.search_records(q, 10, row_offset=b)
                torch.cuda.synchronize()
                print("  shard", i, "records row0:", rec[0, :, 1].tolist(), flush=True)
            print("  got rows0 ", got[1][0].tolist())
            print("  want rows0", w[1][0].tolist())
            print("  got s0 ", got[0][0].tolist())
            print("  want s0", w[0][0].tolist())
