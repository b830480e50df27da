set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_krylov.py -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_krylov.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_krylov.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_comp.json 2> gpurun_out/bench_comp.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_comp.json; tail -3 gpurun_out/bench_comp.err
exit $rc
