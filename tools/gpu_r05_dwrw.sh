#!/bin/bash
# Round 5: register-window dw_fc2 (stage-3 MixFFN back half) — parity tests, then the fused vs unfused timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step test timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "dw_fc2" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_dwfc2.log 2>&1
tail -3 $O/pytest_dwfc2.log
step bench timeout -k 10 200 python tools/dwfc2_bench.py > $O/bench.log 2>&1
cat $O/bench.log
SVK_DWFC2_RW=0 step bench_old timeout -k 10 200 python tools/dwfc2_bench.py > $O/bench_old.log 2>&1
cat $O/bench_old.log
