# round 5: RCCL with peers, two ranks on the one GPU of the box
set -o pipefail
mkdir -p gpurun_out/r5z
timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 scripts/rccl_two_ranks_one_gpu.py > gpurun_out/r5z/log.txt 2>&1; rc=$?
grep -E "rank|Error|error|refused" gpurun_out/r5z/log.txt | grep -v amdgpu.ids | head -20
echo "rc=$rc"
