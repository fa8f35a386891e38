#!/bin/bash
# Round 6: conv data-gradient weight pack (.D) through the tiled transpose — train parity tests, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z4
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "train" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2 3; do for L in new base; do
  if [ $L = base ]; then export SVK_LIB=$PWD/ab/libsvk_base.so; else unset SVK_LIB; fi
  step train$L timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${L}_$i.log 2>&1
  echo "$L run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/train_${L}_$i.log | head -1)"
done; done
