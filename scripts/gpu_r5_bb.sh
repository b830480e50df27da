# round 5: exact float quotients instead of integer divisions in the brick
# kernels' staging / write-out / cell-origin table -- parity, then A/B
# against the previous library (lib/var/r5base.so)
set -o pipefail
mkdir -p gpurun_out/r5bb
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mg.py -k "f64 or f32 or vcycle or resident or deterministic" > gpurun_out/r5bb/pytest.log 2>&1 || { grep -E "Error|error|assert|FAILED" gpurun_out/r5bb/pytest.log | head -20; tail -20 gpurun_out/r5bb/pytest.log; exit 1; }
tail -2 gpurun_out/r5bb/pytest.log
B=dealii-ns-gls_amd/lib/var/r5base.so
for rep in 1 2 3; do
  for lib in new base; do
    if [ $lib = base ]; then export GLS_AMD_LIB=$B; else unset GLS_AMD_LIB; fi
    v=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f64 200 2>/dev/null | tail -1)
    f=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f32 200 2>/dev/null | tail -1)
    c=$(timeout -k 10 120 python3 scripts/prof_vcycle.py 10 2>/dev/null | tail -1)
    echo "$lib $rep | $v | $f | $c"
  done
done | tee gpurun_out/r5bb/ab_idiv.txt
