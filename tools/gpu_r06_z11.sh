#!/bin/bash
# Round 6: the default bench line with the new default step counts (30 timed, 10 warm-up), run twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z16
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
for i in 1; do
  s=$(date +%s)
  step bench timeout -k 10 600 python bench.py > $O/bench_$i.log 2>&1
  echo "run $i: $(( $(date +%s) - s )) s wall, $(grep -o '"value": [0-9.]*' $O/bench_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log | head -1)"
done
