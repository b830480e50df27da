#!/bin/bash
# Time bench.py against every variant library in dealii-ns-gls_amd/lib/var/
# (diagnostic builds: ablations, launch-bound / tiling experiments).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
for so in dealii-ns-gls_amd/lib/var/*.so; do
  v=$(basename "$so" .so)
  GLS_AMD_LIB=$so timeout -k 10 120 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err
  rc=$?
  echo "$v rc=$rc $(python -c "import json,sys;d=json.load(open('gpurun_out/var/$v.json'));print(d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3)" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
