#!/bin/bash
# one GPU call: quick vmult parity of the default library, then an A/B of
# variant libraries (scripts/ab_env.sh) in FP64 at r2 and r3 and FP32 at r2.
#   SPEC="<label> <lib|default> [VAR=value ...]" lines (see ab_env.sh)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NO_PARITY" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py ${PARITY_TESTS} -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/ab_parity.log | tail -3
fi
NREFS="${NREFS_F64:-2 3}" PREC=f64 bash scripts/ab_env.sh | tee gpurun_out/ab_f64.txt
if [ -z "$NO_F32" ]; then
  NREFS=2 PREC=f32 bash scripts/ab_env.sh | tee gpurun_out/ab_f32.txt
fi
