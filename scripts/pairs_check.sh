#!/bin/bash
# layer-pair bricks: parity suite, then bench + rocprof with pairs on / off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pairs
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pairs/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pairs/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pairs/pytest.log | head -20; exit $rc; }
for v in 1 0; do
  GLS_BRICK_PAIRS=$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/pairs/bench_$v.json 2> gpurun_out/pairs/bench_$v.err || exit $?
  GLS_BRICK_PAIRS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pairs/prof_$v -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-companions > gpurun_out/pairs/prof_$v.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/pairs/bench_$v.json'));c=d['companions'];print('pairs=$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], {k:round(v['ms'],4) for k,v in c.items() if isinstance(v,dict) and 'ms' in v})"
  grep -E "k_brick|k_shared" gpurun_out/pairs/prof_$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
