# cold probe with the MALL read-allocation check, then bench.py's default
# line with the read-flush cold companion (and the write flush beside it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6u py:scripts/cold_probe.py:20:4 bench
