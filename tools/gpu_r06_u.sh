#!/bin/bash
# Round 6: 64-query blocks for the resident-K/V attention below 512 queries — parity tests, same-box step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py tests/test_models_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "attention or headline or b2 or b3" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for v in auto 256; do
  if [ $v = auto ]; then unset SVK_ATTN_QB; else export SVK_ATTN_QB=$v; fi
  step bench$v timeout -k 10 200 $B > $O/bench_${v}_$i.log 2>&1
  echo "QB=$v run $i: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log | head -1)"
done; done
