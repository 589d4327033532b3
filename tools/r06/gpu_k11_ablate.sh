#!/bin/bash
# Round 6: where config 2's 39 us go — kernel 11's phase clocks (debug library) and the timing-only
# ablations (RFX_K11_ABLATE bits, wrong results): 2 no row stream, 4 no quantiser, 8 no last-block work,
# 16 no re-score + rank, 32 no bound over the records.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06a}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2> $O/k11_phases.err || { tail -20 $O/k11_phases.err; exit 1; }
cat $O/k11_phases.json
for a in 0 2 4 8 16 32 6 10; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/cfg2_ablate$a.log 2>&1 || { tail -20 $O/cfg2_ablate$a.log; exit 1; }
  echo -n "ablate=$a: "; python3 -c "$S" < $O/cfg2_ablate$a.log
done
