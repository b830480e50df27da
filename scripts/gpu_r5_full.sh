# round 5: the whole GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r5full
timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r5full/pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r5full/pytest.log | head -20; tail -30 gpurun_out/r5full/pytest.log; exit 1; }
tail -2 gpurun_out/r5full/pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r5full/bench.json 2> gpurun_out/r5full/bench.err || { tail -20 gpurun_out/r5full/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5full/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['frac_cold'],d['roofline']['frac_r3'])"
