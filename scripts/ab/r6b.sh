# round 6: stall recovery, dist barrier, wide DCGS2 passes (tests + A/B + GMRES kernel stats)
bash scripts/gpu_run.sh r6b tests::tests/test_gpu_krylov.py,tests/test_gpu_mg.py,tests/test_dist.py,tests/test_gpu_dist_native.py,tests/test_cpp.py,tests/test_amg.py && \
REPS=2 bash scripts/gpu_run.sh r6b abmg:scripts/ab/r6_dcgs.txt && \
bash scripts/gpu_run.sh r6b prof:scripts/prof_gmres.py && \
GLS_GMRES_ORTHO=dcgs-narrow bash scripts/gpu_run.sh r6b_narrow prof:scripts/prof_gmres.py && \
bash scripts/gpu_run.sh r6b py:scripts/dist_projection.py
