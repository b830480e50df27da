#!/bin/bash
# per-dispatch kernel trace of 20 FP32 V-cycles (scripts/prof_vcycle.py):
# which level and kernel the V-cycle time goes to
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vtrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vtrace -o run -- python3 scripts/prof_vcycle.py > gpurun_out/vtrace/log.txt 2>&1
echo "rocprof rc=$?"
