# round 5: kernel + copy trace of threaded in-process group vmults; r3 brick-layer A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5h/trace -o run -- python3 scripts/prof_dist_threaded.py 2 2 20 > gpurun_out/r5h/trace.log 2>&1 || { tail -20 gpurun_out/r5h/trace.log; exit 1; }
grep threaded gpurun_out/r5h/trace.log
bash scripts/gpu_r5_f.sh
