#!/bin/bash
# Round 6: transposed-score attention-backward dQ kernel — parity tests, same-box train A/B, per-kernel times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "train_step" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
for i in 1 2 3; do for v in 1 0; do
  SVK_ATTN_BWD_T=$v step train$v timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${v}_$i.log 2>&1
  echo "ATTN_BWD_T=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/train_${v}_$i.log | head -1)"
done; done
for v in 1 0; do
  SVK_ATTN_BWD_T=$v step prof$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python bench.py --workload train --no-cpu-baseline --steps 10 --warmup 2 > $O/prof$v.log 2>&1
  f=$(find $O/prof$v -name '*kernel_stats.csv' | head -1); grep -E "attn_bwd|wgrad_pk|store_kv" $f | cut -d, -f1-4 | cut -c1-200
done
