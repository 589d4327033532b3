#!/bin/bash
# round 4: the whole GPU suite and smoke on the current build (select a_k count, XCD-balanced kernel 10)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04zf; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['oracle_check']['ok'], d['cpu_baseline']['value'], d['build_id'])"
