# re-entry check after the container was re-created: the rebuilt libraries
# (same sources) through the whole GPU suite, smoke and the driver's bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6r tests smoke bench:--steps:20:--warmup:5
