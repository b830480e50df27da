# one lease: cold probe (with the MALL read-allocation check), the
# non-temporal write-out A/B (r6v.sh), then bench.py's default line with the
# read-flush cold companion
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6u py:scripts/cold_probe.py:20:4 && bash scripts/ab/r6v.sh && \
bash scripts/gpu_run.sh r6u bench
