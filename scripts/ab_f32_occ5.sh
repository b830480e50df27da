set -o pipefail
mkdir -p gpurun_out/v5
for rep in 1 2; do
for cfg in "default 1" "default 0" "v5 0"; do
  set -- $cfg
  if [ $1 = default ]; then L=""; else L="dealii-ns-gls_amd/lib/var/$1.so"; fi
  GLS_PAD32=$2 GLS_AMD_LIB=$L timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-companions --no-parity --precision f32 > gpurun_out/v5/$1_$2_$rep.json 2>/dev/null || exit 1
  echo "$1 pad$2 $rep $(python -c "import json;d=json.load(open('gpurun_out/v5/$1_$2_$rep.json'));print(round(d['ms_per_step']*1e3,2))")"
done; done
