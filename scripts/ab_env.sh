#!/bin/bash
# A/B of library variants with per-variant environments: each line of $SPEC
# is "<label> <lib name or default> [VAR=value ...]"; FP64 vmult at $NREFS,
# alternating, $REPS reps (bench.py without companions / parity)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for nref in ${NREFS:-2}; do
    while read -r label lib envs; do
      [ -z "$label" ] && continue
      if [ "$lib" = default ]; then L=""; else L="dealii-ns-gls_amd/lib/var/$lib.so"; fi
      f=gpurun_out/ab/${label}_${PREC:-f64}_r${nref}_$rep
      env GLS_AMD_LIB=$L $envs timeout -k 10 120 python bench.py --nref $nref --steps ${STEPS:-100} --warmup 20 --no-cpu-baseline --no-companions --no-parity --precision ${PREC:-f64} > $f.json 2> $f.err || { echo "$label failed"; tail -3 $f.err; exit 1; }
      echo "$label ${PREC:-f64} r$nref $rep $(python -c "import json;d=json.load(open('$f.json'));print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))")"
    done <<< "$SPEC"
  done
done
