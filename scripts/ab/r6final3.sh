bash scripts/gpu_run.sh r6final3 bench:--steps:20:--warmup:5 bench stats
