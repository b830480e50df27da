# round 5: curved-brick load placement in the 4-wave FP64 kernel (A/B)
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r5d/pytest.log 2>&1 || { tail -40 gpurun_out/r5d/pytest.log; exit 1; }
tail -2 gpurun_out/r5d/pytest.log
SPEC='new default
geoearly geoearly
clustered default GLS_CURVED_BALANCE=0
r4head r4head
anycart anycart' NREFS='2' REPS=3 bash scripts/ab_env.sh
SPEC='new default
r4head r4head' NREFS='3' REPS=2 bash scripts/ab_env.sh
