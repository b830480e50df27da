#!/bin/bash
# A/B of the default library against dealii-ns-gls_amd/lib/var/<v>.so for
# every v in $VAR (space separated):
# headline FP64 and FP32 vmult, alternating, bench.py without companions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in default ${VAR}; do
    for prec in f64 f32; do
      if [ $lib = default ]; then L=""; else L="dealii-ns-gls_amd/lib/var/$lib.so"; fi
      GLS_AMD_LIB=$L timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-companions --no-parity --precision $prec > gpurun_out/ab/${lib}_${prec}_$rep.json 2> gpurun_out/ab/${lib}_${prec}_$rep.err || exit 1
      echo "$lib $prec $rep $(python -c "import json;d=json.load(open('gpurun_out/ab/${lib}_${prec}_$rep.json'));print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))")"
    done
  done
done
