#!/bin/bash
# fused shared-node reduction (GLS_FUSED_REDUCE=1): parity suite, then
# bench lines with and without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fused
GLS_FUSED_REDUCE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_mg.py tests/test_a_gpu_configs.py tests/test_gpu_krylov.py \
  tests/test_gpu_system_matrix.py tests/test_gpu_outflow.py tests/test_brick_discovery.py tests/test_golden.py \
  > gpurun_out/fused/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/fused/pytest.log; exit 1; }
tail -2 gpurun_out/fused/pytest.log
for f in 0 1; do
  GLS_FUSED_REDUCE=$f timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fused/bench_f$f.json 2> gpurun_out/fused/bench_f$f.err || exit 1
  GLS_FUSED_REDUCE=$f timeout -k 10 120 python bench.py --precision f32 --steps 100 --warmup 10 --no-cpu-baseline --no-companions > gpurun_out/fused/f32_f$f.json 2>/dev/null || exit 1
  python3 - $f <<'PY'
import json, sys
f = sys.argv[1]
d = json.load(open(f"gpurun_out/fused/bench_f{f}.json"))
e = json.load(open(f"gpurun_out/fused/f32_f{f}.json"))
c = d["companions"]
print("fused", f, "f64 us", round(d["ms_per_step"] * 1e3, 2), "kernel", round(d["roofline"]["kernel_ms"] * 1e3, 2),
      "frac", round(d["roofline"]["frac"], 3), "| f32 us", round(e["ms_per_step"] * 1e3, 2),
      "| r3", round(c["r3_f64_warm"]["ms"] * 1e3, 1), "sphere", round(c["sphere_r3_f64_warm"]["ms"] * 1e3, 1),
      "| vcycle", round(c["r2_vcycle_f32_coarse_relax10"]["ms"], 4), "gmres", round(c["r2_gmres_iteration"]["ms"], 4),
      "| cold", round(c["r2_f64_cold"]["ms"] * 1e3, 1))
PY
done
