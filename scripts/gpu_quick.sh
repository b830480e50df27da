#!/bin/bash
# one box session: selected GPU tests (TESTS, default the whole suite), then
# the default bench line (BENCH_ARGS); each step under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest.log | tail -40; tail -3 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  exit $rc
fi
