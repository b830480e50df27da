# round 6 final evidence, part A: the whole GPU suite and smoke()
bash scripts/gpu_run.sh r6final tests smoke
