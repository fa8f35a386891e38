#!/bin/bash
# Round 5: gemm_ln second form (A LDS-DMA ring, W double-buffered) — tests, isolated timing, same-box step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step test timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm_ln" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gln.log 2>&1
tail -1 $O/pytest_gln.log
step bench_gln timeout -k 10 200 python tools/gemm_ln_bench.py > $O/gemm_ln_bench.log 2>&1; grep -v amdgpu.ids $O/gemm_ln_bench.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for v in 1 0 1 0; do
  SVK_GEMM_LN=$v step bench_gln$v timeout -k 10 200 $B > $O/bench_gln$v.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_gln$v.log | head -1 | sed "s/^/gln=$v /"
done
