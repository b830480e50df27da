# round 5: DCGS2 GMRES tests + timing; trace of threaded groups; r3 brick-layer A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests/test_gpu_krylov.py tests/test_gpu_newton.py tests/test_gpu_dist_native.py > gpurun_out/r5i/pytest.log 2>&1 || { tail -40 gpurun_out/r5i/pytest.log; exit 1; }
grep -E "passed|failed|GMRES iterations|threaded" gpurun_out/r5i/pytest.log | tail -8
timeout -k 10 300 python scripts/prof_gmres.py > gpurun_out/r5i/gmres.log 2>&1 || { tail -20 gpurun_out/r5i/gmres.log; exit 1; }
tail -5 gpurun_out/r5i/gmres.log
GLS_GMRES_ORTHO=cgs2 timeout -k 10 300 python scripts/prof_gmres.py > gpurun_out/r5i/gmres_cgs2.log 2>&1 || { tail -20 gpurun_out/r5i/gmres_cgs2.log; exit 1; }
tail -5 gpurun_out/r5i/gmres_cgs2.log
bash scripts/gpu_r5_h.sh
