#!/bin/bash
# the whole GPU suite in one process (per-test timeouts), then smoke() and a
# short bench line; stops at the first failing step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|ERROR" gpurun_out/pytest_all.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-companions --steps 200 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.log || { echo bench failed; tail -5 gpurun_out/bench_short.log; exit 1; }
cat gpurun_out/bench_short.json
