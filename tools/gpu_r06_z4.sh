#!/bin/bash
# Round 6: conv data-gradient weight pack (.D) through the tiled transpose — train parity tests, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z4
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "train" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2 3; do for v in 1 0; do
  SVK_PACK_D_T=$v step train$v timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${v}_$i.log 2>&1
  echo "PACK_D_T=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/train_${v}_$i.log | head -1)"
done; done
