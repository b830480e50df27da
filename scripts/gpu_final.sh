#!/bin/bash
# round-end evidence in one box session: the whole GPU suite, smoke(), the
# default bench line, the rocprofv3 kernel-trace summary of the bench
# command, and kernel stats of the direct-coarse V-cycle and of GMRES(28)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-companions > $O/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vdirect -o run -- python3 scripts/prof_vcycle.py -1 > $O/vdirect.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gmres -o run -- python3 scripts/prof_gmres.py > $O/gmres.log 2>&1
