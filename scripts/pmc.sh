#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --kernel-trace/--pmc only)
# over a short bench run; summaries land in gpurun_out/pmc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 10 --warmup 2 --settle-ms 0 --no-cpu-baseline --no-companions ${BENCH_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($counters) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
FETCH_SIZE
WRITE_SIZE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum
LIST
