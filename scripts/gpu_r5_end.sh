# round 5 end: the whole GPU suite, the default bench line, rocprofv3 stats
# of the bench command (the code as committed)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5end
timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r5end/pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r5end/pytest.log | head -20; tail -30 gpurun_out/r5end/pytest.log; exit 1; }
tail -2 gpurun_out/r5end/pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r5end/bench.json 2> gpurun_out/r5end/bench.err || { tail -20 gpurun_out/r5end/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5end/bench.json'));c=d['companions'];print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['frac_cold'],d['roofline']['frac_r3']);print(c['r2_vcycle_f32_coarse_relax10']['ms'],c['r2_gmres_iteration']['ms'],c['r2_f32_level_warm'].get('ms_back_to_back'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5end/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions > gpurun_out/r5end/bench_stats.json 2> gpurun_out/r5end/bench_stats.err || { tail -5 gpurun_out/r5end/bench_stats.err; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('gpurun_out/r5end/stats/run_kernel_stats.csv')):
    if 'k_brick<3, 2, double' in r[0] or 'shared_reduce_cls<double' in r[0]: print(r[0][:50], r[1], r[3])
"
