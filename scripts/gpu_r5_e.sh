# round 5: padded lattice within the LDS budget + curved-brick load placement (A/B)
set -o pipefail
mkdir -p gpurun_out/r5e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_a_gpu_configs.py > gpurun_out/r5e/pytest.log 2>&1 || { tail -40 gpurun_out/r5e/pytest.log; exit 1; }
tail -2 gpurun_out/r5e/pytest.log
SPEC='new default
geoearly geoearly
r4head r4head' NREFS='2' REPS=5 bash scripts/ab_env.sh
SPEC='new default
r4head r4head' NREFS='3' REPS=2 bash scripts/ab_env.sh
SPEC='new default
r4head r4head' NREFS='2 3' REPS=2 PREC=f32 bash scripts/ab_env.sh
