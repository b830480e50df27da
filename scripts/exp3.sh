#!/bin/bash
# parity subset + bench + phase timeline (stamps build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('vmult us', d['ms_per_step']*1e3, 'kernel us', d['roofline']['kernel_ms']*1e3, 'frac', d['roofline']['frac'])"
if [ -f dealii-ns-gls_amd/lib/var/stamps.so ]; then
GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/stamps.so timeout -k 10 200 python scripts/timeline.py > gpurun_out/tl.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/timeline.json'));print(json.dumps(d['phases_us']));print(d['brick_top_to_rounds_done_us'], d['end_quantiles_us'])"
fi
for so in dealii-ns-gls_amd/lib/var/v_*.so; do
  [ -f "$so" ] || continue
  v=$(basename "$so" .so)
  GLS_AMD_LIB=$so timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$v.json 2> gpurun_out/$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/$v.json'));print('$v', d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3)"
done
if [ "${PROFILE:-0}" = "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'])"
fi
