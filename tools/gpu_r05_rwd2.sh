#!/bin/bash
# Round 5: mixffn_rwd variants (SVK_RW_VAR 3..6) vs mixffn_rw (0): parity + timing, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05rwd2
mkdir -p $O
for v in 5 6; do
  SVK_RW_VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mixffn_rw" > $O/test_$v.log 2>&1 || { echo "tests var $v failed"; tail -30 $O/test_$v.log; exit 1; }
  echo "var $v: $(tail -1 $O/test_$v.log)"
done
for rep in 1 2; do
for v in 0 3 4 5 6; do
  SVK_RW_VAR=$v timeout -k 10 120 python tools/mixffn_prof.py > $O/time_${v}_$rep.txt 2>&1 || { echo "timing var $v failed"; cat $O/time_${v}_$rep.txt; exit 1; }
  echo "var $v: $(tail -1 $O/time_${v}_$rep.txt)"
done
done
