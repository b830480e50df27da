#!/bin/bash
# partitioned path at world 1 (GLS_BENCH_DIST=1): the Python-driven and the
# native distributed multigrid / GMRES beside the single-domain lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dist
GLS_BENCH_DIST=1 timeout -k 10 400 python bench.py --gmres-iteration --no-cpu-baseline --no-companions --steps 20 > gpurun_out/dist/bench_dist_world1.json 2> gpurun_out/dist/bench_dist_world1.err
