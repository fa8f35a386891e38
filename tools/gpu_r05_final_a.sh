#!/bin/bash
# Round-5 closing evidence, part A: the full GPU suite, smoke, and the census of the graph-replayed extraction
# step (launch count, per-kernel time), all into gpurun_out/profiles_r05
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
R=r05
mkdir -p $O/profiles_$R $O/r05c
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
cp $O/pytest_gpu.log $O/profiles_$R/pytest_gpu_full.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r05c/census -o run -- python tools/graph_step_census.py run > $O/r05c/census.log 2>&1
T=$(find $O/r05c/census -name '*kernel_trace.csv' | head -1)
python tools/graph_step_census.py analyse $T --by-kernel --seq $O/profiles_$R/graph_step_sequence.txt > $O/profiles_$R/graph_step_census.txt
head -4 $O/profiles_$R/graph_step_census.txt
