# round 5: threaded in-process groups through gls_dist_vmult (tests + trace),
# one-layer 4-wave vs two-layer 3-wave bricks on the r3 meshes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5g
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests/test_dist.py tests/test_gpu_dist_native.py -k "threaded or local_group_gpu or native_group" > gpurun_out/r5g/pytest.log 2>&1 || { tail -40 gpurun_out/r5g/pytest.log; exit 1; }
grep -E "passed|failed|threaded world" gpurun_out/r5g/pytest.log | tail -12
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5g/trace -o run -- python3 scripts/prof_dist_threaded.py 2 2 20 > gpurun_out/r5g/trace.log 2>&1 || { tail -20 gpurun_out/r5g/trace.log; exit 1; }
tail -2 gpurun_out/r5g/trace.log
bash scripts/gpu_r5_f.sh
