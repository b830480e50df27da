#!/bin/bash
# multigrid-side check: MG / distributed-MG / config GPU tests, then the
# bench (companions incl. the direct-coarse V-cycle), no CPU baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mg
timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py tests/test_dist_mg.py tests/test_a_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mg/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/mg/bench.json 2> gpurun_out/mg/bench.err
