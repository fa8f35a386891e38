#!/bin/bash
# fc1_dwconv pre-activation / wide-C round: parity tests, front-half microbench, same-box train and
# extraction A/Bs.  Output under gpurun_out/fc1dw/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fc1dw; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py \
  -k "fc1_dwconv or unpatchify or patchify or col2im or conv_wgrad_dgrad" > $O/pytest_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 $O/pytest_kernels.log; exit 1; }
tail -3 $O/pytest_kernels.log
timeout -k 10 200 python -u tools/fc1dw_bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_gpu.py \
  > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -30 $O/pytest_train.log; exit 1; }
tail -3 $O/pytest_train.log
for k in 1 2; do
  for e in "SVK_TRAIN_FC1_DWCONV=0 SVK_TRAIN_UNPATCHIFY_SPLIT=0 SVK_TRAIN_COL2IM=0" "SVK_TRAIN_FC1_DWCONV=0 SVK_TRAIN_UNPATCHIFY_SPLIT=0" SVK_TRAIN_FC1_DWCONV=0 SVK_TRAIN_FC1_DWCONV=1 SVK_TRAIN_FC1_DWCONV_C=32,64,128,320,512; do
    v=$(env $e timeout -k 10 300 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline 2>>$O/train_ab.err \
        | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "train $e: $v" | tee -a $O/train_ab.log
  done
done
for k in 1; do
  for e in SVK_FC1_DWCONV_C=32,64,128 SVK_FC1_DWCONV_C=32,64,128,320 SVK_FC1_DWCONV_C=32,64,128,320,512; do
    v=$(env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none 2>>$O/ext_ab.err \
        | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "extract $e: $v" | tee -a $O/ext_ab.log
  done
done
