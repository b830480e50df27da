# PMC passes (one counter group per run) of the x-line DPP kernels (timing
# builds of GLS_XDPP_F32=1 / GLS_XDPP_F64=1, lib/var) beside the product
# library on the same box: SQ_INSTS_LDS per wave, waits, bank conflicts
# (the run needs lib/var: .gpurunignore's lib/var line is lifted for it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r6s
for v in base:f32 x32w4:f32 base:f64 x64w3:f64; do
  lib=${v%%:*}; p=${v#*:}
  L=""; [ "$lib" != base ] && L=dealii-ns-gls_amd/lib/var/$lib.so
  GLS_AMD_LIB=$L NREFS=2 PREC=$p bash scripts/gpu_pmc.sh || exit 1
  D=gpurun_out/pmc_r2; [ "$p" = f32 ] && D=gpurun_out/pmc_f32_r2
  rm -rf gpurun_out/r6s/pmc_${lib}_${p}_r2
  mv $D gpurun_out/r6s/pmc_${lib}_${p}_r2
done
