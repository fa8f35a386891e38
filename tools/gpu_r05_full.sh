#!/bin/bash
# Round-5 evidence session: full GPU suite -> smoke -> extraction profiles + PMC + bench line (tools/gpu_prof.sh,
# R=r05) -> fp32 extraction kernel stats (the fp32 leg's roofline) -> train-step rocprofv3 stats, FETCH/WRITE
# passes and bench line.  Everything lands in gpurun_out/profiles_r05.  A failing step ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
R=r05
mkdir -p $O/profiles_$R
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
if [ -z "$SKIP_SUITE" ]; then
  step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  tail -1 $O/pytest_gpu.log
  cp $O/pytest_gpu.log $O/profiles_$R/pytest_gpu_full.log
fi
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
R=$R bash tools/gpu_prof.sh || exit $?
B="python bench.py --no-cpu-baseline --no-other-workloads"
step prof32 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x32 -o run -- $B --dtype fp32 --other-dtypes none --steps 5 --warmup 2 > $O/prof_x32.log 2>&1
python tools/prof_stats.py $O/prof_x32/run_kernel_stats.csv auto:mean_rows_kernel 40 > $O/profiles_$R/rocprof_extract_fp32_stats.txt
head -3 $O/profiles_$R/rocprof_extract_fp32_stats.txt
step prof_t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t -o run -- $B --workload train --no-graph --steps 5 --warmup 2 > $O/prof_t.log 2>&1
python tools/prof_stats.py $O/prof_t/run_kernel_stats.csv auto:sgd_kernel 45 > $O/profiles_$R/rocprof_train_stats.txt
head -1 $O/profiles_$R/rocprof_train_stats.txt
step pmc_tf timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_tf -o run -- $B --workload train --no-graph --steps 1 --warmup 1 > $O/pmc_tf.log 2>&1
step pmc_tw timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_tw -o run -- $B --workload train --no-graph --steps 1 --warmup 1 > $O/pmc_tw.log 2>&1
cp $O/profiles_$R/pmc_traffic.json $O/pmc_traffic.json
python tools/pmc_traffic.py $O/pmc_tf/run_counter_collection.csv $O/pmc_tw/run_counter_collection.csv $O/pmc_traffic.json train | head -5
cp $O/pmc_traffic.json $O/profiles_$R/pmc_traffic.json
mkdir -p profiles/$R && cp $O/pmc_traffic.json profiles/$R/pmc_traffic.json
step bench_t timeout -k 10 400 python bench.py --workload train --steps 10 --warmup 3 --cpu-baseline-seconds 15 --dump-gemm $O/profiles_$R/train_gemm_shapes.txt > $O/bench_train.log 2>&1
grep '^{' $O/bench_train.log | tail -1 > $O/profiles_$R/bench_train.jsonl
cut -c1-300 $O/profiles_$R/bench_train.jsonl
