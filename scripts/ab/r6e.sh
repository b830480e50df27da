# round 6: DCGS2 dots pass, 2 row halves x 4 column groups vs 8 column groups
bash scripts/gpu_run.sh r6e tests::tests/test_gpu_krylov.py && \
REPS=3 bash scripts/gpu_run.sh r6e abmg:scripts/ab/r6_dots.txt && \
bash scripts/gpu_run.sh r6e prof:scripts/prof_gmres.py
