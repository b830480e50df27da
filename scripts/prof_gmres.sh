#!/bin/bash
# kernel stats of GMRES(28) cycles with the FP32 multigrid (scripts/prof_gmres.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gmres
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gmres -o run -- python3 scripts/prof_gmres.py > gpurun_out/gmres/log.txt 2>&1
