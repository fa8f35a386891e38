#!/bin/bash
# Round 5: BN statistics written, not accumulated (svk_colstats_set: no zero-fill launches in the train step):
# train + temporal train parity, then the train step twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05cs
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_temporal_train_gpu.py > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -60 $O/pytest_train.log; exit 1; }
echo "train: $(tail -1 $O/pytest_train.log)"
B="python bench.py --workload train --no-cpu-baseline --steps 20 --warmup 3"
for rep in 1 2; do
  for v in 1; do
    SVK_NOOP=$v timeout -k 10 300 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "run=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
