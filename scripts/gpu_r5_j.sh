# round 5: deterministic mode + MG/AMG tests after the switch pruning
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_mg.py tests/test_a_gpu_configs.py -k "deterministic or trtri or deferred or coarse_assembly or relaxation_and_vcycle" > gpurun_out/r5j/pytest.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/r5j/pytest.log | head -20; tail -30 gpurun_out/r5j/pytest.log; exit 1; }
grep -E "passed|failed|deterministic|default vs|trtri vs|deferred vs|element vs" gpurun_out/r5j/pytest.log | tail -14
