# round 5: rocprofv3 stats of the bench command; PMC passes FP64 / FP32 at r2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pmc/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions > gpurun_out/r5pmc/bench_stats.json 2> gpurun_out/r5pmc/bench_stats.err || { tail -5 gpurun_out/r5pmc/bench_stats.err; exit 1; }
NREFS=2 PREC=f64 bash scripts/gpu_pmc.sh || exit 1
NREFS=2 PREC=f32 bash scripts/gpu_pmc.sh || exit 1
