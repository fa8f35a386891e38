#!/bin/bash
# dw_fc2_mx timing ablations (SVK_DWFC2_DIAG bits: 1 = W2 of K-step 0 only, 2 = no GELU, 4 = H of K-step 0 only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
for d in 0 1 2 4 7; do
  SVK_DWFC2_DIAG=$d timeout -k 10 120 python tools/dwfc2_bench.py > $O/diag$d.log 2>&1 || { echo "diag $d failed"; exit 1; }
  echo "diag=$d $(grep float16 $O/diag$d.log | head -1)"
done
