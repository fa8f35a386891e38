#!/bin/bash
# Round 5: dw_fc2 (stage-3 MixFFN back half) — parity tests, then fused vs unfused timing (+ SVK_DWFC2_DIAG ablations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step test timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "dw_fc2" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_dwfc2.log 2>&1
tail -1 $O/pytest_dwfc2.log
step bench timeout -k 10 200 python tools/dwfc2_bench.py > $O/bench.log 2>&1
cat $O/bench.log
for d in ${DIAGS:-1 4 5}; do
  SVK_DWFC2_DIAG=$d step diag$d timeout -k 10 120 python tools/dwfc2_bench.py > $O/diag$d.log 2>&1
  echo "diag=$d $(grep float16 $O/diag$d.log | head -1)"
done
