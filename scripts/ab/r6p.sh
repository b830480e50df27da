# Tail reduction (shared-node reduce as tail workgroups of the brick launch):
# vmult parity tests, then alternating A/B against the separate reduce launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6p tests::tests/test_gpu_parity.py,tests/test_a_gpu_configs.py && \
NREFS="2 3" PREC=f64 REPS=3 bash scripts/gpu_run.sh r6p ab:scripts/ab/r6_tail.txt && \
NREFS="2" PREC=f32 REPS=2 bash scripts/gpu_run.sh r6p ab:scripts/ab/r6_tail.txt
