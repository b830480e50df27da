# gls-vmult (the reference's performance.cc on this library): checks, then
# the reference's default (2 5 1) and 3D configurations, timings only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_run.sh r6n 'tests:gls_vmult:tests/test_gls_vmult.py' || exit 1
for cfg in "2 5 1" "2 8 2" "3 4 2" "3 5 1" "3 3 3"; do
  echo "== gls-vmult $cfg" >> gpurun_out/r6n/gls_vmult.txt
  timeout -k 10 300 tools/build/gls-vmult $cfg >> gpurun_out/r6n/gls_vmult.txt 2>&1 || { tail -20 gpurun_out/r6n/gls_vmult.txt; exit 1; }
done
grep -E "==|Number of DoFs|us per vmult" gpurun_out/r6n/gls_vmult.txt
