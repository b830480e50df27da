bash scripts/gpu_run.sh r6final2 tests smoke bench bench:--steps:20:--warmup:5 stats
