#!/bin/bash
# Round 5: stage-4 merged q|kv GEMM (SVK_MERGED_QKV) and the shape-gated gemm_ln (SVK_GEMM_LN=auto):
# model + headline parity, then an interleaved same-box bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_headline_gpu.py > $O/pytest_models.log 2>&1 || { echo "model tests failed"; tail -40 $O/pytest_models.log; exit 1; }
echo "models: $(tail -1 $O/pytest_models.log)"
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for rep in 1 2; do
  for cfg in "1 auto" "0 0"; do
    set -- $cfg
    SVK_MERGED_QKV=$1 SVK_GEMM_LN=$2 timeout -k 10 200 $B > $O/bench_$1_$2_$rep.log 2>&1 || { echo "bench $cfg failed"; tail -20 $O/bench_$1_$2_$rep.log; exit 1; }
    echo "qkv=$1 gln=$2: $(grep -o '"value": [0-9.]*' $O/bench_$1_$2_$rep.log | head -1)"
  done
done
