#!/bin/bash
# One parametrised GPU-box runner for the measurement and evidence steps
# (replaces the per-experiment gpu_r5_*.sh drivers of round 5).
#
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Every step writes under gpurun_out/TAG/, runs under its own time limit, and
# the first failing step ends the run (no GPU step after a failure).  Steps:
#   tests[:KEXPR[:FILES]]  pytest -m gpu (optionally -k KEXPR, on FILES)
#   smoke                  __graft_entry__.smoke()
#   bench[:ARGS]           python bench.py ARGS  -> bench[_N].json
#   stats                  rocprofv3 --kernel-trace --stats of the bench command
#   pmc:f64|f32            PMC passes of the r2 vmult (scripts/gpu_pmc.sh)
#   ab:FILE                alternating A/B of library variants / environments
#                          (scripts/ab_env.sh, SPEC lines from FILE)
#   abmg:FILE              the same for the multigrid (scripts/ab_mg.sh)
#   py:SCRIPT[:ARGS]       python SCRIPT ARGS (colons in ARGS become spaces)
#   prof:SCRIPT[:ARGS]     rocprofv3 --kernel-trace --stats of python SCRIPT ARGS
#                          (prof_NAME/run_kernel_stats.csv)
# The round's profiles/r0N/README.md names the TAG and STEPs of each file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
nb=0
for step in "$@"; do
  kind=${step%%:*}
  arg=
  [ "$kind" != "$step" ] && arg=${step#*:}
  echo "== $step" >&2
  case $kind in
    tests)
      kexpr=${arg%%:*}
      files=tests
      [ "$kexpr" != "$arg" ] && files=$(echo "${arg#*:}" | tr ',' ' ')
      kopt=()
      [ -n "$kexpr" ] && kopt=(-k "$kexpr")
      timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread \
        $files -m gpu "${kopt[@]}" > "$OUT/pytest.log" 2>&1 ||
        { grep -E "FAILED|Error|error" "$OUT/pytest.log" | head -20; tail -30 "$OUT/pytest.log"; exit 1; }
      tail -2 "$OUT/pytest.log"
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ||
        { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log"
      ;;
    bench)
      nb=$((nb + 1))
      f=$OUT/bench_$nb
      timeout -k 10 600 python bench.py ${arg//:/ } > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "
import json; d = json.load(open('$f.json')); r = d['roofline']; c = d.get('companions', {})
print('$f', d['value'], d['ms_per_step'], r['frac'], r.get('frac_cold'), r.get('frac_r3'))
for k in ('r2_f32_level_warm', 'r2_vcycle_f32_coarse_relax10', 'r2_gmres_iteration'):
    if k in c: print('  ', k, {x: y for x, y in c[k].items() if 'ms' in x or 'frac' in x})"
      ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companions \
        > "$OUT/bench_stats.json" 2> "$OUT/bench_stats.err" || { tail -5 "$OUT/bench_stats.err"; exit 1; }
      python3 -c "
import csv
for r in csv.reader(open('$OUT/stats/run_kernel_stats.csv')):
    if 'k_brick<3, 2, double' in r[0] or 'shared_reduce_cls<double' in r[0]: print(r[0][:50], r[1], r[3])"
      ;;
    pmc)
      NREFS=2 PREC=${arg:-f64} bash scripts/gpu_pmc.sh || exit 1
      ;;
    ab)
      SPEC=$(cat "$arg") timeout -k 10 900 bash scripts/ab_env.sh || exit 1
      ;;
    abmg)
      SPEC=$(cat "$arg") timeout -k 10 900 bash scripts/ab_mg.sh || exit 1
      ;;
    py)
      script=${arg%%:*}
      args=
      [ "$script" != "$arg" ] && args=${arg#*:}
      name=$(basename "$script" .py)
      timeout -k 10 400 python3 "$script" ${args//:/ } > "$OUT/$name.txt" 2>&1 ||
        { tail -20 "$OUT/$name.txt"; exit 1; }
      grep -v amdgpu.ids "$OUT/$name.txt" | tail -12
      ;;
    prof)
      script=${arg%%:*}
      args=
      [ "$script" != "$arg" ] && args=${arg#*:}
      name=$(basename "$script" .py)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
        python3 "$script" ${args//:/ } > "$OUT/prof_$name.txt" 2>&1 || { tail -20 "$OUT/prof_$name.txt"; exit 1; }
      grep -v amdgpu.ids "$OUT/prof_$name.txt" | tail -4
      head -12 "$OUT/prof_$name/run_kernel_stats.csv" | cut -c1-160
      ;;
    *)
      echo "unknown step $step" >&2
      exit 2
      ;;
  esac
done
