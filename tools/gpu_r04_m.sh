#!/bin/bash
# In-graph census of the extraction step with the library GEMM policy off / on (same box): per-kernel durations
# inside the replayed graph vs the isolated sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
for v in 0 1; do
  SVK_LIBGEMM=$v step census$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census$v -o run -- python tools/graph_step_census.py run > $O/census$v.log 2>&1
  python tools/graph_step_census.py analyse $(find $O/census$v -name '*kernel_trace.csv' | head -1) --seq $O/seq$v.txt > $O/census$v.txt; cat $O/census$v.txt
done
