# Non-temporal write-out stores (GLS_NT_STORE=1 build, lib/var/nts.so):
# alternating A/B against the product library, FP64 r2 / r3 and FP32 r2
# (the run needs lib/var: .gpurunignore's lib/var line is lifted for it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NREFS="2 3" PREC=f64 REPS=3 bash scripts/gpu_run.sh r6v ab:scripts/ab/r6_nts.txt && \
NREFS="2" PREC=f32 REPS=3 bash scripts/gpu_run.sh r6v ab:scripts/ab/r6_nts.txt
