#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in v3 v2; do
  SVK_LIB=diag_libs/libsvk_$v.so timeout -k 10 200 python -u tools/pk_diag.py > gpurun_out/pkdiag_$v.log 2>&1 || exit 1
  echo "$v done"
done
