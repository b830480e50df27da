#!/bin/bash
# A/B of multigrid-side environments: each line of $SPEC is
# "<label> [VAR=value ...]"; the r0..r2 FP32 V-cycle (direct coarse and 10
# sweeps) and GMRES(28) wall times, alternating, $REPS reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abmg
for rep in $(seq 1 ${REPS:-2}); do
  while read -r label envs; do
    [ -z "$label" ] && continue
    f=gpurun_out/abmg/${label}_$rep
    env $envs timeout -k 10 120 python scripts/prof_vcycle.py -1 > $f.vd 2>&1 || { echo "$label vcycle failed"; tail -3 $f.vd; exit 1; }
    env $envs timeout -k 10 120 python scripts/prof_vcycle.py 10 > $f.v10 2>&1 || { echo "$label vcycle10 failed"; tail -3 $f.v10; exit 1; }
    env $envs timeout -k 10 120 python scripts/prof_gmres.py > $f.g 2>&1 || { echo "$label gmres failed"; tail -3 $f.g; exit 1; }
    echo "$label $rep direct: $(tail -1 $f.vd) | sweeps: $(tail -1 $f.v10) | $(tail -1 $f.g)"
  done <<< "$SPEC"
done
