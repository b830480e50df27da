#!/bin/bash
# A/B of brick-kernel variant libraries (dealii-ns-gls_amd/lib/var/*.so) on
# the headline bench (r2) and the HBM-bound r3: ms per vmult and the
# event-timed kernel time, alternating variants twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in ${VARIANTS:-base pipe sync}; do
    for nref in ${NREFS:-2 3}; do
      GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/$v.so timeout -k 10 180 python bench.py --no-companions --no-cpu-baseline --steps 200 --warmup 20 --nref $nref > gpurun_out/ab/$v.r$nref.$rep.json 2> gpurun_out/ab/$v.r$nref.$rep.log
      rc=$?
      python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab/$v.r$nref.$rep.json'))
print('$v r$nref rep$rep', 'ms %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], 'parity', d['parity']['rel_l2_f64'] if d.get('parity') else None)
" || { echo "$v r$nref rc=$rc"; tail -5 gpurun_out/ab/$v.r$nref.$rep.log; }
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
