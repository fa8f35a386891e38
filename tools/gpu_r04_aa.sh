#!/bin/bash
# Same-box A/B of the XCD-grouped depthwise conv block order (SVK_DW_XCD) on the replayed extraction step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
for r in a b c; do for v in 0 1; do
  SVK_DW_XCD=$v step bench$v$r timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 1500 --warmup 20 > $O/bench_$v$r.log 2>&1
  echo "dw_xcd=$v $(grep -o '"value": [0-9.]*' $O/bench_$v$r.log | head -1)"
done; done
