#!/bin/bash
# Round 6: stage-1 mixffn_rwd with whole-frame strips (SVK_RW_VAR=5, R = 56) vs the 28-row strips (0): kernel
# parity, then isolated timing and the step A/B interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06rw56
mkdir -p $O
SVK_RW_VAR=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mixffn_rw" > $O/test_5.txt 2>&1 || { echo "tests var 5 failed"; tail -30 $O/test_5.txt; exit 1; }
echo "var 5 tests: $(tail -1 $O/test_5.txt)"
for rep in 1 2; do
  for v in 0 5; do
    SVK_RW_VAR=$v timeout -k 10 120 python tools/mixffn_prof.py > $O/time_${v}_$rep.txt 2>&1 || { echo "timing var $v failed"; cat $O/time_${v}_$rep.txt; exit 1; }
    echo "var $v: $(tail -1 $O/time_${v}_$rep.txt)"
  done
done
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for rep in 1 2 3; do
  for v in 0 5; do
    SVK_RW_VAR=$v timeout -k 10 200 $B > $O/bench_${v}_$rep.txt 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.txt; exit 1; }
    echo "rw_var=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.txt | head -1)"
  done
done
