#!/bin/bash
# kernel-level timing of variant libraries (dealii-ns-gls_amd/lib/var/*.so)
# and env settings: rocprofv3 kernel-trace stats of a short bench run per
# combination.  VARS: "name:ENV=val,ENV=val" list (default: each .so, no env)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vprof
COMBOS=${VARS:-$(for so in dealii-ns-gls_amd/lib/var/*.so; do basename $so .so; done)}
for combo in $COMBOS; do
  v=${combo%%:*}; envs=""
  [ "$combo" != "$v" ] && envs=${combo#*:}
  tag=$(echo "$combo" | tr ':,=' '___')
  so=dealii-ns-gls_amd/lib/var/$v.so
  env GLS_AMD_LIB=$so $(echo $envs | tr ',' ' ') timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof/$tag -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-companions --no-parity ${BENCH_ARGS:-} > gpurun_out/vprof/$tag.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -5 gpurun_out/vprof/$tag.log; exit $rc; }
  f=$(find gpurun_out/vprof/$tag -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$tag" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
out=[]
for r in rows:
    n=r["Name"]
    if "k_brick" in n or "k_shared_reduce" in n:
        out.append(f'{n.split("(")[0].replace("void gls::","")[:34]}={float(r["AverageNs"])/1e3:.2f}us(n={r["Calls"]})')
print(sys.argv[2], " ".join(out))
PY
done
