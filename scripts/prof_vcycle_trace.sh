#!/bin/bash
# per-dispatch kernel trace of 20 FP32 V-cycles (scripts/prof_vcycle.py
# $COARSE: 10 sweeps by default, -1 = direct): which level and kernel the
# V-cycle time goes to; output under gpurun_out/${OUT:-vtrace}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-vtrace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 scripts/prof_vcycle.py ${COARSE:-10} > $O/log.txt 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] && python3 scripts/vtrace_summary.py $(find $O -name "*kernel_trace.csv" | head -1) > $O/summary.txt
