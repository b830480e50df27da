bash scripts/gpu_run.sh r6a tests::tests/test_gpu_parity.py,tests/test_a_gpu_configs.py && \
PREC=f32 REPS=2 bash scripts/gpu_run.sh r6a ab:scripts/ab/r6_xdpp.txt && \
PREC=f64 REPS=2 bash scripts/gpu_run.sh r6a ab:scripts/ab/r6_xdpp.txt
