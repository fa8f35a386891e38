#!/bin/bash
# Round 5: mixffn_rwd as the default stage-1 MixFFN: kernel + model parity, then the step A/B against
# the f32-FMA form (SVK_RW_VAR=3), interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05rwd3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "mixffn" tests/test_models_gpu.py tests/test_headline_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for rep in 1 2; do
  for v in 0 3; do
    SVK_RW_VAR=$v timeout -k 10 200 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "rw_var=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
