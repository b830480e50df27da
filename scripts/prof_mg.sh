#!/bin/bash
# rocprofv3 kernel-trace summary of the multigrid companions (setup, V-cycle,
# GMRES iteration) on the headline hierarchy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mgprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mgprof -o run -- python3 scripts/prof_vcycle.py > gpurun_out/mgprof/log.txt 2>&1
echo "rocprof rc=$?"
