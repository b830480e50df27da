bash scripts/gpu_run.sh r6g tests:agglomerated_bottom:tests/test_dist_mg.py py:scripts/host_overhead.py
