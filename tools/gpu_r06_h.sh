#!/bin/bash
# Round 6: where the config-5 chain spends its time beyond the extraction step (rocprofv3 kernel summary of the
# eager e2e step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step prof_e2e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python bench.py --workload e2e --no-cpu-baseline --no-graph --steps 10 --warmup 2 > $O/p.log 2>&1
python tools/prof_stats.py $O/p/run_kernel_stats.csv auto:mean_rows 60 > $O/e2e_stats.txt; cut -c1-200 $O/e2e_stats.txt
