set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_krylov.py tests/test_gpu_mg.py -k "kept_directions or trtri or coarse_gmres_vcycle or relaxation_and_vcycle or gmg_newton" > gpurun_out/r5a/pytest.log 2>&1 || { tail -30 gpurun_out/r5a/pytest.log; exit 1; }
tail -5 gpurun_out/r5a/pytest.log
SPEC='default default
allcart allcart' NREFS='2 3' REPS=2 bash scripts/ab_env.sh
