#!/bin/bash
# distributed-path GPU tests + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_dist.log | tail -15
[ $rc -eq 0 ] || exit $rc
TESTS=tests PROFILE=0 bash scripts/exp3.sh
