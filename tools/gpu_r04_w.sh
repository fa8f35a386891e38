#!/bin/bash
# Gaussian s2d with LDS-DMA staging (SVK_GAUSS_DMA): parity, isolated time, step-start census, same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step tests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_headline_gpu.py -x -q -k "gauss or hc4 or golden or conv2d_s2d_ln or benched_config_fp16 or mit_b3" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for v in 1 0; do
  SVK_STEM_LN16=$v step census$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census$v -o run -- python tools/graph_step_census.py run > $O/census$v.log 2>&1
  python tools/graph_step_census.py analyse $(find $O/census$v -name '*kernel_trace.csv' | head -1) --seq $O/seq$v.txt | tail -2 | cut -c1-90
  head -4 $O/seq$v.txt | cut -c1-80
done
for r in a b; do for v in 0 1; do
  SVK_STEM_LN16=$v step bench$v$r timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 1500 --warmup 20 > $O/bench_$v$r.log 2>&1
  echo "stem_ln=$v $(grep -o '"value": [0-9.]*' $O/bench_$v$r.log | head -1)"
done; done
