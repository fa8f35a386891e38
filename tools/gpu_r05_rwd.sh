#!/bin/bash
# Round 5: stage-1 MixFFN with f16-pair dot-product taps (mixffn_rwd, SVK_RW_VAR=3 at 3 waves/SIMD, 4 at 2)
# against the f32-FMA form (0): parity tests and timing, plus the dot2 / fmac issue-rate microbenchmark
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05rwd
mkdir -p $O
timeout -k 10 60 tools/micro/dot2_rate > $O/dot2_rate.txt 2>&1 || { echo "microbench failed"; exit 1; }
cat $O/dot2_rate.txt
for v in 3 4 0; do
  SVK_RW_VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mixffn_rw" > $O/test_$v.log 2>&1 || { echo "tests var $v failed"; tail -30 $O/test_$v.log; exit 1; }
  echo "var $v: $(tail -1 $O/test_$v.log)"
  SVK_RW_VAR=$v SVK_RW_VERBOSE=1 timeout -k 10 120 python tools/mixffn_prof.py > $O/time_$v.txt 2>&1 || { echo "timing var $v failed"; cat $O/time_$v.txt; exit 1; }
  cat $O/time_$v.txt
done
