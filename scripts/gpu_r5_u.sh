# round 5: resident sweeps against one launch per step with the 5-wave FP32
# per-launch kernels
set -o pipefail
mkdir -p gpurun_out/r5u
SPEC='resident
launches GLS_MG_DEFER=1' REPS=3 timeout -k 10 500 bash scripts/ab_mg.sh | tee gpurun_out/r5u/ab_resident.txt || exit 1
OUT=r5u/vtrace timeout -k 10 330 bash scripts/prof_vcycle_trace.sh && head -14 gpurun_out/r5u/vtrace/summary.txt
