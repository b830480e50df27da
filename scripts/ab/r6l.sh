# timer sections: GPU tests (tally, C++ facade with its report), the
# TimerOutput-style table of a Re3900 r2 GMRES solve, and the roctx ranges
# of the bench command under rocprofv3 --marker-trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6l 'tests:timer or interface or cpp:tests/test_gpu_timer.py,tests/test_gpu_layout.py,tests/test_cpp.py' py:scripts/timer_report.py || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/r6l/marker -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions \
  > gpurun_out/r6l/bench_marker.json 2> gpurun_out/r6l/bench_marker.err || { tail -5 gpurun_out/r6l/bench_marker.err; exit 1; }
ls gpurun_out/r6l/marker
head -5 gpurun_out/r6l/marker/run_marker_api_stats.csv 2>/dev/null || true
