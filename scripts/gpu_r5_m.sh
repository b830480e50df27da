# round 5: phase breakdown of the resident sweeps (timing build)
set -o pipefail
mkdir -p gpurun_out/r5m
timeout -k 10 300 python3 scripts/sweep_timing.py > gpurun_out/r5m/sweep_timing.txt 2>&1; rc=$?
cat gpurun_out/r5m/sweep_timing.txt | head -60
exit $rc
