bash scripts/gpu_run.sh r6k bench:--steps:20:--warmup:5
