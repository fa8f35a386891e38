#!/bin/bash
# Round 5: matrix-core stage-3 dw_fc2 in the extraction step — headline parity, then a same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step head timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py tests/test_models_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_headline.log 2>&1
grep -E "max\|d\||passed|failed" $O/pytest_headline.log | tail -14
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for v in 1 0 1 0; do
  SVK_DWFC2_MX=$v step bench_mx$v timeout -k 10 200 $B > $O/bench_mx$v.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_mx$v.log | head -1 | sed "s/^/mx=$v /"
done
