# round 5: resident smoothing sweeps (k_brick_sweeps) -- parity tests, V-cycle
# A/B against one launch per step, kernel trace of the V-cycle
set -o pipefail
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_mg.py -k "resident or deterministic or deferred or relaxation_and_vcycle" > gpurun_out/r5k/pytest.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/r5k/pytest.log | head -20; tail -30 gpurun_out/r5k/pytest.log; exit 1; }
grep -E "passed|failed|resident|deterministic|default vs|deferred vs" gpurun_out/r5k/pytest.log | tail -14
SPEC='resident
launches GLS_MG_DEFER=1' REPS=2 timeout -k 10 400 bash scripts/ab_mg.sh || exit 1
OUT=r5k/vtrace timeout -k 10 330 bash scripts/prof_vcycle_trace.sh && head -20 gpurun_out/r5k/vtrace/summary.txt
