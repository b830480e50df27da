#!/bin/bash
# PMC passes (scripts/pmc.sh) of the vmult at r2 (headline) and r3 (the
# HBM-bound size), FP64 (PREC=f64, default: gpurun_out/pmc_r2, pmc_r3) or the
# FP32 level operator (PREC=f32: gpurun_out/pmc_f32_r2, pmc_f32_r3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PREC:-f64}
for nref in ${NREFS:-2 3}; do
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--nref $nref --no-parity --precision $P" bash scripts/pmc.sh || exit 1
  python scripts/pmc_summary.py gpurun_out/pmc $nref $P > gpurun_out/pmc/summary.txt || exit 1
  if [ "$P" = f64 ]; then D=gpurun_out/pmc_r$nref; else D=gpurun_out/pmc_${P}_r$nref; fi
  rm -rf $D; mkdir -p $D
  cp gpurun_out/pmc/summary.txt gpurun_out/pmc/traffic.json $D/ 2>/dev/null
  tail -3 $D/summary.txt
done
