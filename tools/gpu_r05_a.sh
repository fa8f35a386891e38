#!/bin/bash
# Round 5: library GEMM removed.  Headline parity (b2 / b3 fp16 / bf16 at B = 256), the GEMM kernel tests,
# the per-shape sweep against torch.matmul (hipBLASLt, yardstick only), then the extraction step with
# gemm_pp off / on, interleaved on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step head timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_headline.log 2>&1
grep -E "max\|d\||passed|failed" $O/pytest_headline.log | tail -12
step gemmtests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or pingpong or persistent" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gemm.log 2>&1
tail -1 $O/pytest_gemm.log
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,60,71 > $O/sweep.log 2>&1
cat $O/sweep.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 400 --warmup 20"
for v in 0 1 0 1; do
  SVK_PP=$v step bench_pp$v timeout -k 10 200 $B > $O/bench_pp$v.log 2>&1
  grep -o '"value": [0-9.]*' $O/bench_pp$v.log | head -1 | sed "s/^/pp=$v /"
done
