#!/bin/bash
# Round 6: the IVF list scan with the register-resident probe selection, against
# the previous build (librfx_base.so): the IVF GPU tests, then config 5 (tools/bench_ivf.py) interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06ivf9}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_cfg5.py tests/test_gpu_ivf_4m.py tests/test_gpu_store_ivf.py tests/test_gpu_sharded.py > $O/pytest_ivf.log 2>&1 || { tail -40 $O/pytest_ivf.log; exit 1; }
tail -1 $O/pytest_ivf.log
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_batch"], d.get("achieved_list_GBps"), d.get("recall_at_k"))'
for i in 1 2; do
  timeout -k 10 600 python -u tools/bench_ivf.py > $O/ivf_new_$i.log 2>&1 || { tail -20 $O/ivf_new_$i.log; exit 1; }
  echo -n "new $i: "; python3 -c "$S" < $O/ivf_new_$i.log
  RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 600 python -u tools/bench_ivf.py > $O/ivf_base_$i.log 2>&1 || { tail -20 $O/ivf_base_$i.log; exit 1; }
  echo -n "base $i: "; python3 -c "$S" < $O/ivf_base_$i.log
done
