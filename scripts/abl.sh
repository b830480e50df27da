#!/bin/bash
# Diagnostic: time the ablation builds (make abl) of the apply kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 4 8 14}; do
  if [ "$v" = "0" ]; then lib=dealii-ns-gls_amd/lib/libglsamd.so; else lib=dealii-ns-gls_amd/lib/abl/libglsamd_abl$v.so; fi
  GLS_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abl_$v.json 2>/dev/null
  rc=$?
  [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/abl_$v.json'));print('abl $v', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
