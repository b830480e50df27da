#!/bin/bash
# PMC passes (scripts/pmc.sh) of the headline r2 and the HBM-bound r3 vmult,
# summaries under gpurun_out/pmc_r2, gpurun_out/pmc_r3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for nref in ${NREFS:-2 3}; do
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--nref $nref --no-parity" bash scripts/pmc.sh || exit 1
  python scripts/pmc_summary.py gpurun_out/pmc $nref f64 > gpurun_out/pmc/summary.txt || exit 1
  rm -rf gpurun_out/pmc_r$nref; mkdir -p gpurun_out/pmc_r$nref
  cp gpurun_out/pmc/summary.txt gpurun_out/pmc/traffic.json gpurun_out/pmc_r$nref/ 2>/dev/null
  tail -3 gpurun_out/pmc_r$nref/summary.txt
done
