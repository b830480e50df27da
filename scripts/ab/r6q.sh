# Tail reduction: where the time goes (release fence per brick, write-through
# slot stores, the flag waits), alternating at r2 FP64; then the parity gate of
# the fence-free variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NREFS="2" PREC=f64 REPS=2 bash scripts/gpu_run.sh r6q ab:scripts/ab/r6_tail2.txt && \
GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/nofence.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions > gpurun_out/r6q/nofence_parity.json 2> gpurun_out/r6q/nofence_parity.err && \
python -c "import json; d=json.load(open('gpurun_out/r6q/nofence_parity.json')); print(d['ms_per_step'], d.get('parity'))"
