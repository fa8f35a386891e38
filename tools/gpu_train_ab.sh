#!/bin/bash
# Train-step round: parity tests of the new backward pieces, the train-step GPU suite, and a same-box
# interleaved A/B of the switches.  Output under gpurun_out/trainab/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trainab; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_gpu.py \
  tests/test_kernels_gpu.py -k "train or col2im or unpatchify or patchify or fc1_dwconv or conv" > $O/pytest.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OFF="SVK_TRAIN_FC1_DWCONV=0 SVK_TRAIN_UNPATCHIFY_SPLIT=0 SVK_TRAIN_COL2IM=0 SVK_PACK_TRANSPOSE=0"
for e in "$OFF" SVK_NONE=1 "$OFF" SVK_NONE=1 SVK_TRAIN_COL2IM=0 SVK_TRAIN_UNPATCHIFY_SPLIT=0 SVK_PACK_TRANSPOSE=0 SVK_TRAIN_FC1_DWCONV=0; do
  v=$(env $e timeout -k 10 300 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline 2>>$O/train_ab.err \
      | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "train $e: $v" | tee -a $O/train_ab.log
done
