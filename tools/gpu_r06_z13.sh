#!/bin/bash
# Round 6, last code state: the full GPU suite and smoke once more (the wgrad split target and the bench step counts
# changed after the closing bundle)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z17
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu_full.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
