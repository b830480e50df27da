#!/bin/bash
# round-end evidence (one box session): the whole GPU suite, the default
# bench line (CPU baseline + companions), the rocprofv3 kernel-trace summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_all.log | tail -5; tail -2 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-companions > gpurun_out/prof.log 2>&1
echo "rocprof rc=$?"
