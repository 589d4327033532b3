"""GPU: the N > 1 bench step end to end, rehearsed with 2 ranks sharing the one GPU (gloo exchange,
`--one-device`): row shards, per-rank two-pass search to records, the exchange, the gathered merge,
max-over-ranks timing and the JSON line — and rank 0's oracle check of the gathered answer against
oracle.search.topk_blocks over ALL rows (regenerated from the counter-based generator), plus
`--check` (the sharded answer equals one whole-index search).  Runs bench.py as child processes
(torch.distributed.run), never exec."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("rows,extra", [(300_000, []), (100_000, ["--nq", "1", "--dtype", "f32"])])
def test_two_rank_bench_step_is_oracle_checked(rows, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--one-device", "--check", "--no-cpu-baseline",
           "--rows", str(rows), "--steps", "3", "--warmup", "1"] + extra
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["value"] > 0
    oc = d["oracle_check"]
    assert oc["ok"] and oc["answer"] == "gathered merge (rank 0)" and oc["rows"] == rows
    assert "check ok" in p.stdout
