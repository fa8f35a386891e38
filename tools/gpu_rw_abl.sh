#!/bin/bash
# mixffn_rw timing ablations (SVK_RW_DIAG: 1 = no per-row barrier, 2 = ReLU for GELU) x variants (SVK_RW_VAR)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARS:-0 1 2 3}; do for d in ${DIAGS:-0 1 2 3}; do
  echo -n "var=$v diag=$d: "
  SVK_RW_VAR=$v SVK_RW_DIAG=$d timeout -k 5 60 python tools/mixffn_bench.py --only rw --reps 20 2>&1 | grep "C=64" || exit 1
done; done
