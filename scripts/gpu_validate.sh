set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v1/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/v1/bench.json 2> gpurun_out/v1/bench.err
