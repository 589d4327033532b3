#!/bin/bash
# Round 6: kernel 11 A/B against the previous build (librfx_base.so), interleaved on one box: config 2,
# kernel 11's tests first and a PMC FETCH_SIZE pass of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/${1:-gpurun_out/r06k11}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen_valu.py tests/test_gpu_screen.py tests/test_gpu_sharded.py tests/test_gpu_filters.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
C2="--rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $C2 > $O/cfg2_new_$i.log 2>&1 || { tail -20 $O/cfg2_new_$i.log; exit 1; }
  echo -n "new $i: "; python3 -c "$S" < $O/cfg2_new_$i.log
  RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py $C2 > $O/cfg2_base_$i.log 2>&1 || { tail -20 $O/cfg2_base_$i.log; exit 1; }
  echo -n "base $i: "; python3 -c "$S" < $O/cfg2_base_$i.log
done
cd /tmp
P2="--rows 100000 --dtype f32 --nq 1 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_new -o pmc_new -- python $R/bench.py $P2 > $O/bench_pmc_new.log 2>&1 || { tail -20 $O/bench_pmc_new.log; exit 1; }
RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_base -o pmc_base -- python $R/bench.py $P2 > $O/bench_pmc_base.log 2>&1 || { tail -20 $O/bench_pmc_base.log; exit 1; }
python3 - <<PY
import csv
for n in ("new", "base"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open("$O/pmc_%s/pmc_%s_counter_collection.csv" % (n, n))) if "screen_valu_kernel" in r["Kernel_Name"]]
    print(n, "FETCH bytes per launch (x2 KB)", 2 * 1024 * sum(v) / len(v), "ratio to 76.9 MB", 2 * 1024 * sum(v) / len(v) / (100000 * 768 + 100000 / 32 * 16))
PY
