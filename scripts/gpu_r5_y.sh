# round 5 timing experiment: the shared-node reduce launched twice per vmult
# (lib/var/reduce2x.so): the second launch reads partials the first left in
# its XCD's L2 -- an upper bound for an XCD-aware reduce order
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5y
GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/reduce2x.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5y/t -o run -- python3 scripts/time_vmult.py input_hoffmann_3D_Re3900.json 2 f64 100 > gpurun_out/r5y/log.txt 2>&1 || { tail -3 gpurun_out/r5y/log.txt; exit 1; }
python3 - <<'PY'
import csv, glob, statistics as st
f = glob.glob('gpurun_out/r5y/t/*kernel_trace.csv')[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
first, second, brick, gap1, gap2 = [], [], [], [], []
for i, r in enumerate(rows):
    if 'k_brick<3, 2, double' in r['Kernel_Name'] and i + 2 < len(rows):
        a, b = rows[i + 1], rows[i + 2]
        if 'shared_reduce' in a['Kernel_Name'] and 'shared_reduce' in b['Kernel_Name']:
            d = lambda x: int(x['End_Timestamp']) - int(x['Start_Timestamp'])
            brick.append(d(r)); first.append(d(a)); second.append(d(b))
            gap1.append(int(a['Start_Timestamp']) - int(r['End_Timestamp']))
            gap2.append(int(b['Start_Timestamp']) - int(a['End_Timestamp']))
print(f"{len(first)} vmults: brick {st.median(brick)/1e3:.2f} us, reduce after brick {st.median(first)/1e3:.2f} us (gap {st.median(gap1)/1e3:.2f}), same reduce again {st.median(second)/1e3:.2f} us (gap {st.median(gap2)/1e3:.2f})")
PY
