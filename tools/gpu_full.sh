#!/bin/bash
# Full GPU session: all GPU tests -> smoke -> rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE PMC
# passes (extraction and training) -> pmc_traffic.json -> bench lines (extraction with cpu_baseline, training).
# Every GPU step has its own time limit; the script stops at the first step that fails.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
B="python bench.py --no-cpu-baseline"
step prof_x timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x -o run -- $B --steps 5 --warmup 2 > $O/prof_x.log 2>&1
step pmc_xf timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_xf -o run -- $B --steps 2 --warmup 1 > $O/pmc_xf.log 2>&1
step pmc_xw timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_xw -o run -- $B --steps 2 --warmup 1 > $O/pmc_xw.log 2>&1
step prof_t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t -o run -- $B --workload train --no-graph --steps 5 --warmup 2 > $O/prof_t.log 2>&1
step pmc_tf timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_tf -o run -- $B --workload train --no-graph --steps 2 --warmup 1 > $O/pmc_tf.log 2>&1
step pmc_tw timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_tw -o run -- $B --workload train --no-graph --steps 2 --warmup 1 > $O/pmc_tw.log 2>&1
rm -f $O/pmc_traffic.json
python tools/pmc_traffic.py $O/pmc_xf/run_counter_collection.csv $O/pmc_xw/run_counter_collection.csv $O/pmc_traffic.json extract > /dev/null
python tools/pmc_traffic.py $O/pmc_tf/run_counter_collection.csv $O/pmc_tw/run_counter_collection.csv $O/pmc_traffic.json train > /dev/null
cp $O/pmc_traffic.json profiles/r01/pmc_traffic.json
step bench_x timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 > $O/bench_extract.log 2>&1
tail -1 $O/bench_extract.log | cut -c1-600
step bench_t timeout -k 10 300 python bench.py --workload train --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > $O/bench_train.log 2>&1
tail -1 $O/bench_train.log | cut -c1-600
# widened rows: CausalMambaModel (selective scan) and the frame transform
step prof_m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_m -o run -- $B --workload mamba --steps 2 --warmup 1 > $O/prof_m.log 2>&1
step prof_p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p -o run -- $B --workload preproc --steps 5 --warmup 1 > $O/prof_p.log 2>&1
step bench_m timeout -k 10 200 python bench.py --workload mamba --steps 3 --warmup 1 --cpu-baseline-seconds 15 > $O/bench_mamba.log 2>&1
tail -1 $O/bench_mamba.log | cut -c1-300
step bench_p timeout -k 10 200 python bench.py --workload preproc --steps 10 --warmup 2 --cpu-baseline-seconds 10 > $O/bench_preproc.log 2>&1
tail -1 $O/bench_preproc.log | cut -c1-300
