#!/bin/bash
# round 5: SQ counters of the shipped kernel 10 (production = per-tile barrier + publish on change, and
# its MODE 1 and 512; round 4's schedule, MODE 0 / 9, for reference) at 10M rows and at the 8-GPU shard
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r; mkdir -p $O
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
C="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_MFMA_MOPS_I8"
cd /tmp
for size in 10m shard; do
  if [ $size = 10m ]; then ROWS=10000000; V=1010485760,1010485761,800000009,1010486272; else ROWS=1250000; V=1010485760,1010485761,1010486272,800000000; fi
  for p in A B C; do
    timeout -s KILL 150 rocprofv3 --pmc ${!p} --output-format csv -d $O/pmc_${size}_$p -o pmc -- python3 $R/tools/k10_variants.py --rows $ROWS --rounds 1 --burst 5 --variants $V > $O/run_${size}_$p.log 2>&1 || { echo "pass $size $p failed"; tail -5 $O/run_${size}_$p.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $O/pmc_${size}_*/pmc_counter_collection.csv --kernel scan_screen --json $O/pmc_${size}.json > $O/pmc_${size}.txt || exit 1
  grep -E "^_Z|/" $O/pmc_${size}.txt
done
