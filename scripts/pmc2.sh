#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per pass), plus the
# counter list of the box.  Summaries: gpurun_out/pmc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($counters) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU
FETCH_SIZE
WRITE_SIZE
TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TCC_HIT_sum TCC_MISS_sum
LIST
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1
tail -60 gpurun_out/pmc/summary.txt
