#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
for v in 1 0; do
  SVK_PP=$v timeout -k 10 300 python -u -m pytest tests/test_headline_gpu.py -q -rf -s -k "b3_fp16 or b2_fp16 or config5" --timeout 250 --timeout-method thread -p no:cacheprovider > $O/head_pp$v.log 2>&1; echo "head pp=$v rc=$?"
  grep -E "fp16 B=256|passed|failed|chain" $O/head_pp$v.log | head -8
done
step bench timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-other-workloads --no-cpu-baseline > $O/bench.log 2>&1
grep '^{' $O/bench.log | cut -c1-600
step bench_pp0 env SVK_PP=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-other-workloads --no-cpu-baseline > $O/bench_pp0.log 2>&1
grep '^{' $O/bench_pp0.log | cut -c1-300
step train timeout -k 10 400 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline --no-other-workloads --dump-gemm $O/train_gemm_shapes.txt > $O/bench_train.log 2>&1
grep '^{' $O/bench_train.log | cut -c1-300
head -40 $O/train_gemm_shapes.txt
