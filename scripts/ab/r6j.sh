# host-wait modes vs the fixed cost of a timed region (scripts/sync_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r6j
for m in auto spin yield auto; do
  timeout -k 10 300 python3 scripts/sync_probe.py $m >> gpurun_out/r6j/sync_probe.txt 2>> gpurun_out/r6j/sync_probe.err || exit 1
done
cat gpurun_out/r6j/sync_probe.txt
