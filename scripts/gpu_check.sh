#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace
# summary.  Every GPU step has its own time limit; the script stops at the
# first crash / timeout (exit codes other than 0 = pass, 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
TESTS=${TESTS:-tests}
timeout -k 10 900 python -m pytest $TESTS -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
exit 0
