#!/bin/bash
# GPU evidence run: the GPU test suite, the bench line (companions, CPU
# baseline), rocprofv3 kernel stats of the bench command; outputs under
# gpurun_out/$TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-check}
mkdir -p $T
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest_gpu.log 2>&1
  rc=$?; tail -3 $T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $T/bench.json 2> $T/bench.err || { tail -5 $T/bench.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench.json'));print(d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['frac'], d['parity']['ok']); c=d.get('companions') or {}; [print(k, {kk: (round(vv,4) if isinstance(vv,float) else vv) for kk,vv in v.items() if kk in ('ms','roofline_frac','back_to_back_ms','back_to_back_frac')}) for k,v in c.items() if isinstance(v,dict)]"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions > $T/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp "$f" $T/kernel_stats.csv; head -8 $T/kernel_stats.csv | cut -c1-200
if [ -n "$AB_SPEC" ]; then
  SPEC="$AB_SPEC" NREFS="${AB_NREFS:-2 3}" REPS=${AB_REPS:-2} bash scripts/ab_env.sh 2>&1 | tee $T/ab.txt
fi
