#!/bin/bash
# occupancy variants, split sweep, r3 throughput
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=50 bash scripts/variants.sh || exit $?
SPLITS="0 128 256 512" bash scripts/split_sweep.sh || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --nref 3 > gpurun_out/r3.json 2> gpurun_out/r3.err || exit $?
cat gpurun_out/r3.json
