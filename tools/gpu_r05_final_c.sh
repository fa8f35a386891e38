#!/bin/bash
# Round-5 closing evidence, part C (after the last train-step changes): full GPU suite, smoke, train-step
# rocprofv3 summary, and the default bench line, into gpurun_out/profiles_r05c
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
P=$O/profiles_r05c
mkdir -p $P
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $P/pytest_gpu_full.log 2>&1
tail -1 $P/pytest_gpu_full.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1
tail -1 $P/smoke.log
step prof_t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tc -o run -- python bench.py --no-cpu-baseline --no-other-workloads --workload train --no-graph --steps 5 --warmup 2 > $O/prof_tc.log 2>&1
python tools/prof_stats.py $O/prof_tc/run_kernel_stats.csv auto:sgd_kernel 45 > $P/rocprof_train_stats.txt
head -1 $P/rocprof_train_stats.txt
step bench timeout -k 10 400 python bench.py > $P/bench_default.log 2>&1
grep '^{' $P/bench_default.log | tail -1 > $P/bench_default.json
cut -c1-300 $P/bench_default.json
