#!/bin/bash
# Round 6: where the runtime copy / fill kernels sit in the eager train step (census), plus the train step's
# rocprof summary at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step trace timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --workload train --no-graph --steps 3 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1
python tools/train_copy_census.py $(find $O/tr -name '*kernel_trace.csv' | head -1) > $O/copy_census.txt; head -80 $O/copy_census.txt | cut -c1-330
