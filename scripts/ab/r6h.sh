bash scripts/gpu_run.sh r6h py:scripts/clock_probe.py py:scripts/host_overhead.py
