#!/bin/bash
# GMRES-side check: Krylov / Newton / layout / C++ facade GPU tests, then the
# bench companions (no CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kry
timeout -k 10 300 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_newton.py tests/test_gpu_layout.py tests/test_cpp.py tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kry/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/kry/bench.json 2> gpurun_out/kry/bench.err
