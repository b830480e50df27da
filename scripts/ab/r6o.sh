# Upper bound of recomputing U / grad U in the kernel: the FP64 vmult with
# those 12 table fields not streamed (timing-only GLS_EXP_NO_UGU build),
# alternating against the product library at r2 and r3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NREFS="2 3" PREC=f64 REPS=3 bash scripts/gpu_run.sh r6o ab:scripts/ab/r6_ugu.txt
