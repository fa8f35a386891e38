#!/bin/bash
# Profile collection for the extraction headline (fp16) -> gpurun_out/profiles_$R (copied into profiles/$R): rocprofv3 kernel-trace stats of the
# benched (graph-replayed) step, FETCH_SIZE / WRITE_SIZE passes (HBM bytes per launch) and an MFMA-busy
# pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) on the eager step; every pass its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${R:-r03}
mkdir -p gpurun_out/profiles_$R
export TMPDIR=/tmp
O=gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
W=${W:-extract}
DT=${DT:-fp16}
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --workload $W --dtype $DT"
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o run -- $B --steps 10 --warmup 2 > $O/prof_$W.log 2>&1
python tools/prof_stats.py $O/prof_$W/run_kernel_stats.csv auto:mean_rows_kernel 45 > $O/profiles_$R/rocprof_${W}_${DT}_stats.txt
cp $O/prof_$W/run_kernel_stats.csv $O/profiles_$R/rocprof_${W}_${DT}_kernel_stats.csv
tail -1 $O/prof_$W.log | cut -c1-300
python tools/trace_gaps.py $O/prof_$W/run_kernel_trace.csv 2600 | tee $O/profiles_$R/trace_gaps_${W}_${DT}.txt
step pmc_f timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${W}_f -o run -- $B --no-graph --steps 1 --warmup 1 > $O/pmc_${W}_f.log 2>&1
step pmc_w timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${W}_w -o run -- $B --no-graph --steps 1 --warmup 1 > $O/pmc_${W}_w.log 2>&1
step pmc_m timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${W}_m -o run -- $B --no-graph --steps 1 --warmup 1 > $O/pmc_${W}_m.log 2>&1
cp profiles/$R/pmc_traffic.json $O/pmc_traffic.json 2>/dev/null
python tools/pmc_traffic.py $O/pmc_${W}_f/run_counter_collection.csv $O/pmc_${W}_w/run_counter_collection.csv $O/pmc_traffic.json $W | head -12
cp $O/pmc_traffic.json $O/profiles_$R/pmc_traffic.json
cp profiles/$R/pmc_mfma.json $O/pmc_mfma.json 2>/dev/null
python tools/pmc_mfma.py $O/pmc_${W}_m/run_counter_collection.csv $O/pmc_mfma.json ${W}_${DT} 1 "${DOM:-gemm_pk<_Float16, PkCfg<128, 128}" "${DOMFLOP:-0}"
cp $O/pmc_mfma.json $O/profiles_$R/pmc_mfma.json
# this round's counters are the ones the bench line quotes (bench.py reads the newest profiles/rNN)
mkdir -p profiles/$R && cp $O/pmc_traffic.json $O/pmc_mfma.json profiles/$R/
mkdir -p $O/profiles_$R/pmc
for p in f w m; do gzip -c $O/pmc_${W}_$p/run_counter_collection.csv > $O/profiles_$R/pmc/${W}_${DT}_$p.csv.gz; done
step bench timeout -k 10 300 python bench.py --workload $W --dtype $DT --steps 20 --warmup 5 > $O/bench_${W}.log 2>&1
grep "^{" $O/bench_${W}.log | tail -1 > $O/profiles_$R/bench_${W}_${DT}.json
cut -c1-600 $O/profiles_$R/bench_${W}_${DT}.json
