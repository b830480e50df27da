# round 5: resident sweeps' timeout path forced (spin bound 0) -> counted and
# NaN; the default library's resident tests again
set -o pipefail
mkdir -p gpurun_out/r5dd
GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/spin0.so timeout -k 10 120 python3 scripts/sweep_timeout_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5dd/spin0.txt
timeout -k 10 120 python3 scripts/sweep_timeout_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5dd/default.txt || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_mg.py -k "resident or deterministic or deferred" > gpurun_out/r5dd/pytest.log 2>&1 || { tail -20 gpurun_out/r5dd/pytest.log; exit 1; }
tail -2 gpurun_out/r5dd/pytest.log
