#!/bin/bash
# Round 5: the DropPath masks in one launch (svk_keep_mask_multi): kernel + train parity, then the train-step A
# (SVK_TRAIN_MASK_MULTI=0: one keep_mask launch per mask), interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05km
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "keep_mask" > $O/pytest_k.log 2>&1 || { echo "kernel tests failed"; tail -40 $O/pytest_k.log; exit 1; }
echo "kernel: $(tail -1 $O/pytest_k.log)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_temporal_train_gpu.py > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -60 $O/pytest_train.log; exit 1; }
echo "train: $(tail -1 $O/pytest_train.log)"
B="python bench.py --workload train --no-cpu-baseline --steps 20 --warmup 3"
for rep in 1 2; do
  for v in 1 0; do
    SVK_TRAIN_MASK_MULTI=$v timeout -k 10 300 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "mask_multi=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
