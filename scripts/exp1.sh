#!/bin/bash
# tail/latency experiment: k_brick time vs number of bricks launched, and r3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/variants.sh || exit $?
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --nref 3 > gpurun_out/r3.json 2> gpurun_out/r3.err || exit $?
cat gpurun_out/r3.json
