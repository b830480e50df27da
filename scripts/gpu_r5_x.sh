# round 5: shared-node reduce with one thread per node (both 16-byte packs)
# against one thread per pack (lib/var/reduce1.so), FP64 r2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
for rep in 1 2; do
  for lib in default reduce1; do
    if [ $lib = reduce1 ]; then export GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/reduce1.so; else unset GLS_AMD_LIB; fi
    rm -rf gpurun_out/r5x/$lib$rep
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5x/$lib$rep -o run -- python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f64 200 > gpurun_out/r5x/$lib$rep.log 2>&1 || { tail -3 gpurun_out/r5x/$lib$rep.log; exit 1; }
    f=$(find gpurun_out/r5x/$lib$rep -name "*kernel_stats.csv" | head -1)
    echo "$lib $rep: $(grep -v amdgpu gpurun_out/r5x/$lib$rep.log | grep r2 | tail -1) | reduce $(grep -m1 shared_reduce $f | awk -F, '{print $(NF-4)}') ns | brick $(grep -m1 'k_brick<3, 2, double' $f | awk -F, '{print $(NF-4)}') ns"
  done
done | tee gpurun_out/r5x/summary.txt
GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/reduce1.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('reduce1 parity',d['parity'])"
