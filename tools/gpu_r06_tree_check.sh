#!/bin/bash
# Round 6: the committed tree's library (with the SVK_RW_VAR=5 instantiation added after the closing bundle): full
# GPU suite, smoke and the default bench line once more
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06tc
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_full.txt 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $O/pytest_gpu_full.txt)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
echo "smoke: $(tail -1 $O/smoke.txt)"
timeout -k 10 600 python bench.py > $O/bench.txt 2>&1 || { echo "bench failed"; tail -20 $O/bench.txt; exit 1; }
grep '^{' $O/bench.txt | tail -1 > $O/bench_default.json; cut -c1-200 $O/bench_default.json
