#!/bin/bash
# Round 6: re-check of two off-by-default switches on today's build, same box: SVK_PP=1 (256x256 ping-pong GEMM by
# policy) on the extraction step, SVK_TRAIN_DWFC_FWD=1 on the train step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z10
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for v in 0 1; do
  SVK_PP=$v step pp$v timeout -k 10 200 $B > $O/pp_${v}_$i.log 2>&1
  echo "PP=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/pp_${v}_$i.log | head -1)"
done; done
for i in 1 2; do for v in 0 1; do
  SVK_TRAIN_DWFC_FWD=$v step t$v timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/t_${v}_$i.log 2>&1
  echo "TRAIN_DWFC_FWD=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/t_${v}_$i.log | head -1)"
done; done
