#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py for every variant library in
# dealii-ns-gls_amd/lib/var/ (diagnostic builds); prints per-kernel averages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vprof
for so in dealii-ns-gls_amd/lib/var/*.so; do
  v=$(basename "$so" .so)
  GLS_AMD_LIB=$so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof/$v -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/vprof/$v.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  f=$(find gpurun_out/vprof/$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
out=[]
for r in rows:
    n=r["Name"]
    if "k_brick" in n or "k_shared_reduce" in n:
        out.append(f'{n.split("(")[0].replace("void gls::","")[:40]}={float(r["AverageNs"])/1e3:.2f}us')
print(sys.argv[2], " ".join(out))
PY
done
