#!/bin/bash
# Round 5: same-box A/B of the gemm_pk SGPR-base DMA addressing (SVK_LIB = the library built without it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
PREV=deep-learning-for-surgical-video-analysis_amd/svk/libsvk_prev.so
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 300 --warmup 20"
for v in new prev new prev; do
  if [ $v = prev ]; then export SVK_LIB=$PREV; else unset SVK_LIB; fi
  timeout -k 10 200 $B > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' $O/bench_$v.log | head -1)"
done
unset SVK_LIB
for v in new prev; do
  if [ $v = prev ]; then export SVK_LIB=$PREV; else unset SVK_LIB; fi
  timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_$v.log 2>&1 || { echo "train $v failed"; exit 1; }
  echo "train $v $(grep -o '"value": [0-9.]*' $O/train_$v.log | head -1)"
done
