#!/bin/bash
# Round 5: wide-tile GEMM (gemm_wt) correctness + per-shape sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step wttest timeout -k 10 150 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wide_tile" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_wt.log 2>&1
tail -3 $O/pytest_wt.log
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,90,91,92,93 > $O/sweep.log 2>&1
cat $O/sweep.log
