#!/bin/bash
# Round 5: the head's resizes in one launch (SVK_RESIZE_MULTI) + the short-K GEMM tile sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05rs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "resize" > $O/pytest_resize.log 2>&1 || { echo "resize tests failed"; tail -40 $O/pytest_resize.log; exit 1; }
echo "resize: $(tail -1 $O/pytest_resize.log)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_headline_gpu.py > $O/pytest_models.log 2>&1 || { echo "model tests failed"; tail -40 $O/pytest_models.log; exit 1; }
echo "models: $(tail -1 $O/pytest_models.log)"
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for rep in 1 2; do
  for v in 1 0; do
    SVK_RESIZE_MULTI=$v timeout -k 10 200 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "resize_multi=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
timeout -k 10 400 python tools/pk_cfg_sweep.py --cfgs=-1,10,20,30,40,60 --reps 30 > $O/sweep.txt 2>&1 || { echo "sweep failed"; tail $O/sweep.txt; exit 1; }
