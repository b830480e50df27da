# round 6: stall recovery, agglomeration, dist barrier, C++ Newton, AMG default (tests); L2 table prefetch A/B
bash scripts/gpu_run.sh r6c tests::tests/test_gpu_krylov.py,tests/test_gpu_mg.py,tests/test_dist.py,tests/test_gpu_dist_native.py,tests/test_cpp.py,tests/test_amg.py && \
PREC=f64 REPS=3 bash scripts/gpu_run.sh r6c ab:scripts/ab/r6_pf.txt && \
PREC=f32 REPS=3 bash scripts/gpu_run.sh r6c ab:scripts/ab/r6_pf.txt
