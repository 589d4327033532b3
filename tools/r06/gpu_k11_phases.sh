#!/bin/bash
# Round 6: kernel 11's phase clocks (debug library) and timing ablations on the current build, config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06ph}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2> $O/k11_phases.err || { tail -20 $O/k11_phases.err; exit 1; }
grep -v amdgpu $O/k11_phases.json
for a in 0 2 8 16 10; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/cfg2_ablate$a.log 2>&1 || { tail -20 $O/cfg2_ablate$a.log; exit 1; }
  echo -n "ablate=$a: "; python3 -c "$S" < $O/cfg2_ablate$a.log
done
