# round 5: resident sweeps with tagged-granule hand-offs -- parity, A/B, phases
set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_mg.py -k "resident or deterministic or deferred" > gpurun_out/r5n/pytest.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/r5n/pytest.log | head -20; tail -30 gpurun_out/r5n/pytest.log; exit 1; }
grep -E "passed|failed|resident|deterministic|default vs|deferred vs" gpurun_out/r5n/pytest.log | tail -8
SPEC='resident
launches GLS_MG_DEFER=1' REPS=2 timeout -k 10 400 bash scripts/ab_mg.sh || exit 1
OUT=r5n/vtrace timeout -k 10 330 bash scripts/prof_vcycle_trace.sh && head -6 gpurun_out/r5n/vtrace/summary.txt || exit 1
timeout -k 10 300 python3 scripts/sweep_timing.py > gpurun_out/r5n/sweep_timing.txt 2>&1; rc=$?
head -40 gpurun_out/r5n/sweep_timing.txt
exit $rc
