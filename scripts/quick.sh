#!/bin/bash
# parity tests of the operator + brick-size sweep of the bench (one box session)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_dist.py} -m gpu -x -q > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/bricks_sweep.sh
