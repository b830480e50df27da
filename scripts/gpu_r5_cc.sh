# round 5: FP32 sweep buffers of 83 instead of 107 packs per cell (same
# modelled conflicts), two-layer FP32 bricks at 5 waves, 11x12 lattice for
# one-layer FP32 -- parity, then A/B against lib/var/r5base.so
set -o pipefail
mkdir -p gpurun_out/r5cc
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mg.py tests/test_sphere.py tests/test_dist.py -m gpu > gpurun_out/r5cc/pytest.log 2>&1 || { grep -E "Error|error|assert|FAILED" gpurun_out/r5cc/pytest.log | head -20; tail -20 gpurun_out/r5cc/pytest.log; exit 1; }
tail -2 gpurun_out/r5cc/pytest.log
B=dealii-ns-gls_amd/lib/var/r5base.so
for rep in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export GLS_AMD_LIB=$B; else unset GLS_AMD_LIB; fi
    a=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f32 200 2>/dev/null | tail -1 | cut -d' ' -f2-4)
    b=$(timeout -k 10 120 python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 3 f32 30 2>/dev/null | tail -1 | cut -d' ' -f2-4)
    c=$(timeout -k 10 150 python3 scripts/time_vmult.py input_sphere_amg.json 3 f32 20 2>/dev/null | tail -1 | cut -d' ' -f2-4)
    d=$(timeout -k 10 120 python3 scripts/prof_vcycle.py 10 2>/dev/null | tail -1)
    echo "$lib $rep | Re3900 $a | Re3900 $b | sphere $c | $d"
  done
done | tee gpurun_out/r5cc/ab.txt
