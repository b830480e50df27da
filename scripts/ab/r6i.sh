bash scripts/gpu_run.sh r6i py:scripts/clock_probe.py:0,100,300,1000,3000
