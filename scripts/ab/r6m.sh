# final validation after the timer sections: whole GPU suite, smoke, the
# driver's bench command, and the partitioned path at world 1 (settle included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6m tests smoke bench:--steps:20:--warmup:5 || exit 1
GLS_BENCH_DIST=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions \
  > gpurun_out/r6m/bench_dist1.json 2> gpurun_out/r6m/bench_dist1.err || { tail -20 gpurun_out/r6m/bench_dist1.err; exit 1; }
python3 -c "
import json; d = json.load(open('gpurun_out/r6m/bench_dist1.json'))
print('dist world 1', d['value'], d['ms_per_step'], d.get('settle'), d['config']['parallelism'], d.get('native_exchange_check'))"
