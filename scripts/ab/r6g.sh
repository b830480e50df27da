bash scripts/gpu_run.sh r6g 'tests:agglomerated_bottom or interface:tests/test_dist_mg.py,tests/test_gpu_layout.py' py:scripts/host_overhead.py
