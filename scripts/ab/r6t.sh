# cold-flush probe (write vs read flush of the MALL), then the x-line PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6t py:scripts/cold_probe.py:20:4 && bash scripts/ab/r6s.sh
