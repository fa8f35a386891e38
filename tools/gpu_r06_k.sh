#!/bin/bash
# Round 6: extended-epilogue tile policy (64 x 64 / 128 x 64) — GEMM / train parity tests, then a same-box train A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or train or backward or grad" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
for i in 1 2 3; do for v in 1 0; do
  SVK_PK_EXT_POLICY=$v step train$v timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${v}_$i.log 2>&1
  echo "EXT_POLICY=$v run $i: $(grep -o '"value": [0-9.]*' $O/train_${v}_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/train_${v}_$i.log | head -1)"
done; done
