#!/bin/bash
# Round 5: gemm_ln (proj / shared MLP + residual + norm in one kernel) — tests, headline parity, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step test timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm_ln or dw_fc2" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gln.log 2>&1
tail -1 $O/pytest_gln.log
step bench_dw timeout -k 10 200 python tools/dwfc2_bench.py > $O/dwfc2_bench.log 2>&1; grep float $O/dwfc2_bench.log
step head timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py tests/test_models_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_headline.log 2>&1
grep -E "max\|d\||passed|failed" $O/pytest_headline.log | tail -8
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for v in 1 0 1 0; do
  SVK_GEMM_LN=$v step bench_gln$v timeout -k 10 200 $B > $O/bench_gln$v.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_gln$v.log | head -1 | sed "s/^/gln=$v /"
done
for v in "14,7,28" "14,7" "14,7,28" "14,7"; do
  SVK_DWFC2_MX_WIDTHS=$v step bench_w28 timeout -k 10 200 $B > $O/bench_w28.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_w28.log | head -1 | sed "s/^/mx_widths=$v /"
done
for v in 1 0 1 0; do
  SVK_EARLY_STEM=$v step bench_es$v timeout -k 10 200 $B > $O/bench_es$v.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_es$v.log | head -1 | sed "s/^/early_stem=$v /"
done
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run > $O/census.log 2>&1
T=$(find $O/census -name '*kernel_trace.csv' | head -1)
python tools/graph_step_census.py analyse $T --by-kernel --seq $O/census_seq.txt > $O/census.txt; head -4 $O/census.txt; head -8 $O/census_seq.txt
