# round 5: FP32 one-layer brick kernels at 5 waves (per-geometry bodies, no
# relaxation-operand prefetch) -- parity, then A/B against the previous
# library (lib/var/r5base.so)
set -o pipefail
mkdir -p gpurun_out/r5r
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mg.py -k "f32 or vcycle or relaxation or smooth or level" > gpurun_out/r5r/pytest.log 2>&1 || { grep -E "Error|error|assert|FAILED" gpurun_out/r5r/pytest.log | head -20; tail -20 gpurun_out/r5r/pytest.log; exit 1; }
tail -2 gpurun_out/r5r/pytest.log
B=dealii-ns-gls_amd/lib/var/r5base.so
for rep in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export GLS_AMD_LIB=$B; else unset GLS_AMD_LIB; fi
    v=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f32 100 2>/dev/null | tail -1)
    v3=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 3 f32 30 2>/dev/null | tail -1)
    c=$(timeout -k 10 120 python3 scripts/prof_vcycle.py 10 2>/dev/null | tail -1)
    g=$(timeout -k 10 120 python3 scripts/prof_gmres.py 2>/dev/null | tail -1)
    echo "$lib $rep | $v | $v3 | $c | $g"
  done
done | tee gpurun_out/r5r/ab_f32_five_waves.txt
