#!/bin/bash
# Round-6 closing evidence: full GPU suite, smoke, the default bench line, rocprofv3 kernel summaries of the
# headline (b2 fp16), the callers' model (b3 fp16 / fp32) and the train step, the replayed-step census with the
# critical path, and the counter passes scoped to the replayed graph steps.  Output: gpurun_out/r06z
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06ze
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
if [ -z "$SKIP_PYTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_full.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu_full.log
  case $rc in 0|1) ;; *) exit $rc;; esac
  step b3prec timeout -k 10 300 python -u -m pytest tests/test_headline_gpu.py -m gpu -q -s -p no:cacheprovider -k "b3 or benched_config_fp16" > $O/pytest_b3_precision.log 2>&1
  grep -i "logit\|b3\|fp16" $O/pytest_b3_precision.log | head -8
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
fi
step bench timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1
grep '^{' $O/bench_default.log | tail -1 > $O/bench_default.json
cut -c1-300 $O/bench_default.json
step prof_x timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x -o run -- python bench.py --no-cpu-baseline --no-other-workloads --other-dtypes none --steps 20 --warmup 3 > $O/prof_x.log 2>&1
python tools/prof_stats.py $O/prof_x/run_kernel_stats.csv auto:mean_rows 40 > $O/rocprof_extract_fp16_stats.txt; head -3 $O/rocprof_extract_fp16_stats.txt
step prof_b3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b3 -o run -- python bench.py --variant mit_b3_evp --no-cpu-baseline --no-other-workloads --other-dtypes none --steps 20 --warmup 3 > $O/prof_b3.log 2>&1
python tools/prof_stats.py $O/prof_b3/run_kernel_stats.csv auto:mean_rows 40 > $O/rocprof_extract_b3_fp16_stats.txt; head -3 $O/rocprof_extract_b3_fp16_stats.txt
step prof_b3f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b3f -o run -- python bench.py --variant mit_b3_evp --dtype fp32 --no-cpu-baseline --no-other-workloads --other-dtypes none --steps 6 --warmup 2 > $O/prof_b3f.log 2>&1
python tools/prof_stats.py $O/prof_b3f/run_kernel_stats.csv auto:mean_rows 40 > $O/rocprof_extract_b3_fp32_stats.txt; head -3 $O/rocprof_extract_b3_fp32_stats.txt
step prof_t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t -o run -- python bench.py --workload train --no-cpu-baseline --no-graph --steps 5 --warmup 2 > $O/prof_t.log 2>&1
python tools/prof_stats.py $O/prof_t/run_kernel_stats.csv auto:sgd_kernel 45 > $O/rocprof_train_stats.txt; head -3 $O/rocprof_train_stats.txt
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run --replays 6 > $O/census.log 2>&1
T=$(find $O/census -name '*kernel_trace.csv' | head -1)
python tools/graph_step_census.py analyse $T --by-kernel --seq $O/graph_step_sequence.txt > $O/graph_step_census.txt; sed -n 8,12p $O/graph_step_census.txt
step pmc_m timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_m -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_m.log 2>&1
step pmc_f timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_f.log 2>&1
step pmc_w timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_w.log 2>&1
python tools/pmc_mfma.py $(find $O/pmc_m -name '*counter_collection.csv' | head -1) $O/pmc_mfma.json extract_fp16 6 --graph
python tools/pmc_traffic.py $(find $O/pmc_f -name '*counter_collection.csv' | head -1) $(find $O/pmc_w -name '*counter_collection.csv' | head -1) $O/pmc_traffic.json extract 6 | head -4
gzip -f $(find $O/pmc_m $O/pmc_f $O/pmc_w -name '*counter_collection.csv')
rm -rf $O/prof_x $O/prof_b3 $O/prof_b3f $O/prof_t $O/census
