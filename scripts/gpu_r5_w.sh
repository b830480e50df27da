# round 5: bench line with the resident-sweep statistics; kernel statistics
# of five GMRES(28) cycles
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 600 python bench.py > gpurun_out/r5w/bench.json 2> gpurun_out/r5w/bench.err || { tail -20 gpurun_out/r5w/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5w/bench.json'));c=d['companions'];print(d['value'],d['ms_per_step'],d['roofline']['frac']);print(c['r2_vcycle_f32_coarse_relax10']);print(c['r2_gmres_iteration']['ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5w/gmres -o run -- python3 scripts/prof_gmres.py > gpurun_out/r5w/gmres.log 2>&1 || { tail -5 gpurun_out/r5w/gmres.log; exit 1; }
tail -2 gpurun_out/r5w/gmres.log
head -16 $(find gpurun_out/r5w/gmres -name "*kernel_stats.csv" | head -1) | cut -d, -f1-5
