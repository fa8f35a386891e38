#!/bin/bash
# Round 5: kernel census of the graph-replayed b2 extraction step (launch count, per-kernel time in the replay),
# and the train step's rocprof summary after the column-sum fix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run > $O/census.log 2>&1
T=$(find $O/census -name '*kernel_trace.csv' | head -1)
python tools/graph_step_census.py analyse $T --by-kernel --seq $O/census_seq.txt > $O/census.txt; head -4 $O/census.txt; sed -n '/per replayed step/,+25p' $O/census.txt
step train timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t -o run -- python bench.py --workload train --steps 12 --warmup 3 --no-cpu-baseline > $O/train.log 2>&1
python tools/prof_stats.py $O/prof_t/run_kernel_stats.csv auto:sgd_kernel 45 > $O/train_stats.txt
head -12 $O/train_stats.txt
grep -o '"value": [0-9.]*' $O/train.log | head -1
