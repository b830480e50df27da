# round 5 final evidence: the whole GPU suite, the default bench line,
# rocprofv3 stats of the bench command, PMC of the FP64 and FP32 r2 kernels,
# resident-sweep phase timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5final
timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r5final/pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r5final/pytest.log | head -20; tail -30 gpurun_out/r5final/pytest.log; exit 1; }
tail -2 gpurun_out/r5final/pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r5final/bench.json 2> gpurun_out/r5final/bench.err || { tail -20 gpurun_out/r5final/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5final/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['frac_cold'],d['roofline']['frac_r3'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5final/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions > gpurun_out/r5final/bench_stats.json 2> gpurun_out/r5final/bench_stats.err || { tail -5 gpurun_out/r5final/bench_stats.err; exit 1; }
NREFS=2 PREC=f64 bash scripts/gpu_pmc.sh || exit 1
NREFS=2 PREC=f32 bash scripts/gpu_pmc.sh || exit 1
timeout -k 10 300 python3 scripts/sweep_timing.py > gpurun_out/r5final/sweep_timing.txt 2>&1 || exit 1
tail -12 gpurun_out/r5final/sweep_timing.txt
