#!/bin/bash
# PMC passes + summary for the default bench workload (r2, f64)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc 2 f64 > gpurun_out/pmc/summary.txt || exit $?
tail -1 gpurun_out/pmc/summary.txt
