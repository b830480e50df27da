# final validation of the round (after the cold-flush change): whole GPU suite,
# smoke, the driver's bench command, and rocprofv3 statistics of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6x tests smoke bench:--steps:20:--warmup:5 stats
