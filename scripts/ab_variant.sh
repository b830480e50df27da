#!/bin/bash
# A/B of the default library against dealii-ns-gls_amd/lib/var/<v>.so for
# every v in $VAR (space separated), alternating, bench.py without
# companions: $PRECS (default "f64 f32") x $NREFS (default "2") x $REPS reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for nref in ${NREFS:-2}; do
  for lib in default ${VAR}; do
    for prec in ${PRECS:-f64 f32}; do
      if [ $lib = default ]; then L=""; else L="dealii-ns-gls_amd/lib/var/$lib.so"; fi
      f=gpurun_out/ab/${lib}_${prec}_r${nref}_$rep
      GLS_AMD_LIB=$L timeout -k 10 120 python bench.py --nref $nref --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --no-companions --no-parity --precision $prec > $f.json 2> $f.err || exit 1
      echo "$lib $prec r$nref $rep $(python -c "import json;d=json.load(open('$f.json'));print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))")"
    done
  done
  done
done
