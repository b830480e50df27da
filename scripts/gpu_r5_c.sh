# round 5: A/B of the 4-wave FP64 brick kernels (spill-free) against the round-4 library
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r5c/pytest.log 2>&1 || { tail -40 gpurun_out/r5c/pytest.log; exit 1; }
tail -2 gpurun_out/r5c/pytest.log
SPEC='new default
r4head r4head
anycart anycart' NREFS='2 3' REPS=3 bash scripts/ab_env.sh
