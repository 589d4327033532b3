#!/bin/bash
# round 5: kernel 10 publishing a list's best only when it rose (debug kModePubOnChange, scratch library
# librfx_dbg_pub.so; variant encoding 10^8 RING + MODE) against production; the 8-GPU shard step's PMC
# traffic and kernel-trace summary; kernel 11's phases; then the whole -m gpu suite on the shipped build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05k; mkdir -p $O
V=1002097152,1010485760,1002097664
RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_dbg_pub.so timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_pub_shard.txt 2>&1 || { tail -20 $O/k10_pub_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_pub_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
grep '"variant"' $O/k10_pub_shard.txt
RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_dbg_pub.so timeout -k 10 500 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_pub_10m.txt 2>&1 || { tail -20 $O/k10_pub_10m.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_pub_10m.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
grep '"variant"' $O/k10_pub_10m.txt
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | head -30
cd /tmp
Ps="--rows 1250000 --force-comm --steps 20 --warmup 2 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcfs -o pmcfs -- python $R/bench.py $Ps > $O/bench_pmcfs.log 2>&1 || { tail -20 $O/bench_pmcfs.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcws -o pmcws -- python $R/bench.py $Ps > $O/bench_pmcws.log 2>&1 || { tail -20 $O/bench_pmcws.log; exit 1; }
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -60 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
