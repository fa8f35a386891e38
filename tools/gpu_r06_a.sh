#!/bin/bash
# Round 6, first GPU call: GPU suite after the diag/ADVICE changes, the default bench line (now with the mit_b3
# legs), the replayed-step census with the critical-path figure, the counter passes scoped to the replayed
# graph steps (pmc_mfma / pmc_traffic --graph), and the GEMM tile sweep + ablations (diagnostic library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
[ -n "$SKIP_PYTEST" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac   # test failures: go on; a crash / timeout: stop
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,60,80,82,84,100 --shapes "s3 fc1,head,s4 fc2,s4 fc1,s2 fc2,s3 fc2,s4 kv" > $O/sweep.txt 2>&1
cat $O/sweep.txt | grep -v amdgpu.ids | cut -c1-400
for d in 0 1 2 4 8 12; do
  SVK_LIB=$PWD/deep-learning-for-surgical-video-analysis_amd/svk/libsvk_diag.so SVK_PK_DIAG=$d step diag$d timeout -k 10 120 python tools/pk_cfg_sweep.py --cfgs 60 --rounds 3 --shapes "s3 fc1,head" > $O/diag$d.txt 2>&1
  echo "diag=$d: $(grep -v amdgpu.ids $O/diag$d.txt | cut -c1-120 | tr '\n' ' ')"
done
step bench timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1
grep '^{' $O/bench_default.log | tail -1 > $O/bench_default.json
cut -c1-200 $O/bench_default.json
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run --replays 6 > $O/census.log 2>&1
T=$(find $O/census -name '*kernel_trace.csv' | head -1)
python tools/graph_step_census.py analyse $T --by-kernel --seq $O/census_seq.txt > $O/census.txt; sed -n 1,12p $O/census.txt
step pmc_m timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_m -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_m.log 2>&1
step pmc_f timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_f.log 2>&1
step pmc_w timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o p --output-format csv -- python tools/graph_step_census.py run --replays 6 > $O/pmc_w.log 2>&1
python tools/pmc_mfma.py $(find $O/pmc_m -name '*counter_collection.csv' | head -1) $O/pmc_mfma.json extract_fp16 6 --graph
python tools/pmc_traffic.py $(find $O/pmc_f -name '*counter_collection.csv' | head -1) $(find $O/pmc_w -name '*counter_collection.csv' | head -1) $O/pmc_traffic.json extract 6 | head -8
