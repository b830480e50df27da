# round 5: k_brick time against the number of bricks launched (first N of
# the r2 launch order; timing only, variant build lib/var/exp_nb.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
for nb in 1600 1280 1024 768 512 256; do
  GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/exp_nb.so GLS_EXP_NB=$nb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5q/nb$nb -o run -- python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f64 100 > gpurun_out/r5q/nb$nb.log 2>&1 || { tail -5 gpurun_out/r5q/nb$nb.log; exit 1; }
  f=$(find gpurun_out/r5q/nb$nb -name "*kernel_stats.csv" | head -1)
  echo "nb $nb: $(grep -m1 'k_brick' $f | cut -c1-200)"
done | tee gpurun_out/r5q/summary.txt
