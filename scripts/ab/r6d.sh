# round 6: wide DCGS2 passes (A/B + GMRES kernel stats), per-rank projection to 2/4/8 GPUs
REPS=2 bash scripts/gpu_run.sh r6d abmg:scripts/ab/r6_dcgs.txt && \
bash scripts/gpu_run.sh r6d prof:scripts/prof_gmres.py && \
GLS_GMRES_ORTHO=dcgs-narrow bash scripts/gpu_run.sh r6d_narrow prof:scripts/prof_gmres.py && \
bash scripts/gpu_run.sh r6d py:scripts/dist_projection.py && \
GLS_BENCH_DIST=1 bash scripts/gpu_run.sh r6d_dist1 bench:--gmres-iteration:--no-cpu-baseline:--steps:20
