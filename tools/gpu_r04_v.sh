#!/bin/bash
# bf16 library-GEMM policy (SVK_LIBGEMM=2) on the train step: parity of the benched B = 88 step, then a same-box
# A/B of the graph-replayed train step and of the bf16 extraction step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
SVK_LIBGEMM=2 step tests timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_headline_gpu.py -x -q -k "b88 or bf16" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for r in a b; do for v in 1 2; do
  SVK_LIBGEMM=$v step train$v$r timeout -k 10 200 python bench.py --workload train --no-cpu-baseline --no-other-workloads --steps 100 --warmup 5 > $O/train_$v$r.log 2>&1
  echo "train lib=$v $(grep -o '"value": [0-9.]*' $O/train_$v$r.log | head -1)"
  SVK_LIBGEMM=$v step ext$v$r timeout -k 10 200 python bench.py --dtype bf16 --other-dtypes none --no-cpu-baseline --no-other-workloads --steps 500 --warmup 10 > $O/ext_$v$r.log 2>&1
  echo "bf16 extract lib=$v $(grep -o '"value": [0-9.]*' $O/ext_$v$r.log | head -1)"
done; done
