# round 5: resident sweeps with sc1 slot loads (no acquire) -- parity + A/B
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_mg.py -k "resident or deterministic" > gpurun_out/r5l/pytest.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/r5l/pytest.log | head -20; tail -30 gpurun_out/r5l/pytest.log; exit 1; }
grep -E "passed|failed|resident|deterministic|default vs" gpurun_out/r5l/pytest.log | tail -8
SPEC='resident
launches GLS_MG_DEFER=1' REPS=2 timeout -k 10 400 bash scripts/ab_mg.sh || exit 1
OUT=r5l/vtrace timeout -k 10 330 bash scripts/prof_vcycle_trace.sh && head -6 gpurun_out/r5l/vtrace/summary.txt
