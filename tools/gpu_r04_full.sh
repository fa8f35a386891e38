#!/bin/bash
# Round-4 full GPU suite + smoke (regression check at HEAD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04full
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -15 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|Error" | head -20
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
timeout -k 10 300 python -u tools/conv_bench.py > $O/conv_bench.log 2>&1; echo "conv_bench rc=$?"
grep -v amdgpu.ids $O/conv_bench.log | head -4
