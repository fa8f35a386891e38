#!/bin/bash
# Round 5: the frozen DWConv + fc1 data gradient as one matrix-core kernel in the train step
# (SVK_TRAIN_DWFC_BWD): kernel + train parity, then the train-step A/B interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05db
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "dw_fc2" > $O/pytest_k.log 2>&1 || { echo "kernel tests failed"; tail -40 $O/pytest_k.log; exit 1; }
echo "kernel: $(tail -1 $O/pytest_k.log)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_temporal_train_gpu.py > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -60 $O/pytest_train.log; exit 1; }
echo "train: $(tail -1 $O/pytest_train.log)"
B="python bench.py --workload train --no-cpu-baseline --steps 20 --warmup 3"
for rep in 1 2; do
  for v in 1 0; do
    SVK_TRAIN_DWFC_BWD=$v timeout -k 10 300 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "dwfc_bwd=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
