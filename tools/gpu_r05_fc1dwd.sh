#!/bin/bash
# Round 5: the stage-2 front half with the pair window (fc1dw_rwd, default; SVK_RW_VAR=3 the f32-FMA form,
# 4 the pair form at 3 waves per SIMD): parity, kernel timing, step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05fd
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "fc1_dwconv" > $O/pytest_k.log 2>&1 || { echo "kernel tests failed"; tail -40 $O/pytest_k.log; exit 1; }
echo "kernel: $(tail -1 $O/pytest_k.log)"
for rep in 1 2; do
  for v in 0 3 4; do
    SVK_RW_VAR=$v timeout -k 10 120 python tools/fc1dw_prof.py > $O/time_${v}_$rep.txt 2>&1 || { echo "timing $v failed"; cat $O/time_${v}_$rep.txt; exit 1; }
    echo "var $v: $(tail -1 $O/time_${v}_$rep.txt)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_headline_gpu.py > $O/pytest_models.log 2>&1 || { echo "model tests failed"; tail -40 $O/pytest_models.log; exit 1; }
echo "models: $(tail -1 $O/pytest_models.log)"
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for rep in 1 2; do
  for v in 0 3; do
    SVK_RW_VAR=$v timeout -k 10 200 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "rw_var=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
