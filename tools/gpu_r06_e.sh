#!/bin/bash
# Round 6: training-forward dw_fc2_mx (pre-activation store + DropPath row scale) and the attention-backward
# accumulator zeroing inside the dQ kernel: parity tests, train-step A/B, the step's runtime-kernel census
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "dw_fc2 or attention_bwd or train" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2; do for v in 0 1; do
  SVK_TRAIN_DWFC_FWD=$v step train$v timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${v}_$i.log 2>&1
  echo "DWFC_FWD=$v run $i: $(grep -o '"value": [0-9.]*' $O/train_${v}_$i.log | head -1)"
done; done
step trace timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --workload train --no-graph --steps 3 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1
python tools/train_copy_census.py $(find $O/tr -name '*kernel_trace.csv' | head -1) > $O/copy_census.txt; head -3 $O/copy_census.txt | cut -c1-300
