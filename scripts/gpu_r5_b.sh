# round 5: parity of the 4-wave FP64 brick kernels + A/B against the round-4 library
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_a_gpu_configs.py tests/test_brick_discovery.py > gpurun_out/r5b/pytest.log 2>&1 || { tail -40 gpurun_out/r5b/pytest.log; exit 1; }
tail -3 gpurun_out/r5b/pytest.log
SPEC='new default
r4head r4head' NREFS='2 3' REPS=3 bash scripts/ab_env.sh
