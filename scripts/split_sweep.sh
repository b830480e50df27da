#!/bin/bash
# tail experiment: time the vmult vs the number of trailing bricks split in halves
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/split
for sp in ${SPLITS:-0 64 128 256 384 512 768 1600}; do
  GLS_BRICK_SPLIT=$sp timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/split/$sp.json 2> gpurun_out/split/$sp.err || exit $?
  echo "split $sp $(python -c "import json;d=json.load(open('gpurun_out/split/$sp.json'));print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))")"
done
