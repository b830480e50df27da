#!/bin/bash
# FP32 level-operator experiments: occupancy variants and trailing-brick
# splits (diagnostic; one box session)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/f32
export TMPDIR=/tmp
B="--precision f32 --steps 100 --warmup 10 --no-cpu-baseline --no-companions"
ms() { python -c "import json;d=json.load(open('$1'));print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"; }
timeout -k 10 120 python bench.py $B > gpurun_out/f32/base.json 2>/dev/null || exit $?
echo "base $(ms gpurun_out/f32/base.json)"
for v in occ32_4 occ32_5; do
  GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/$v.so timeout -k 10 120 python bench.py $B > gpurun_out/f32/$v.json 2>/dev/null || exit $?
  echo "$v $(ms gpurun_out/f32/$v.json)"
  GLS_PAD32=0 GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/$v.so timeout -k 10 120 python bench.py $B > gpurun_out/f32/${v}_nopad.json 2>/dev/null || exit $?
  echo "$v nopad $(ms gpurun_out/f32/${v}_nopad.json)"
done
GLS_PAD32=0 timeout -k 10 120 python bench.py $B > gpurun_out/f32/base_nopad.json 2>/dev/null || exit $?
echo "base nopad $(ms gpurun_out/f32/base_nopad.json)"
for sp in 0 224 448 800 1600; do
  GLS_BRICK_SPLIT=$sp timeout -k 10 120 python bench.py $B > gpurun_out/f32/split$sp.json 2>/dev/null || exit $?
  echo "split$sp $(ms gpurun_out/f32/split$sp.json)"
done
for sp in 0 256 512; do
  GLS_BRICK_SPLIT=$sp timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-companions > gpurun_out/f32/f64split$sp.json 2>/dev/null || exit $?
  echo "f64 split$sp $(ms gpurun_out/f32/f64split$sp.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32/prof -o run -- python3 bench.py $B --steps 20 > gpurun_out/f32/prof.log 2>&1
echo "rocprof rc=$?"
