#!/bin/bash
# kernel stats of 20 FP32 V-cycles with the deck's direct coarse solver
# (free-dof inverse GEMV), after the multigrid tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vdirect
timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vdirect/pytest.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vdirect -o run -- python3 scripts/prof_vcycle.py -1 > gpurun_out/vdirect/log.txt 2>&1
