#!/bin/bash
# gemm_pp (256-row ping-pong GEMM) iteration: parity tests, then the tile sweep against hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04pp
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pptest timeout -k 10 150 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "pingpong" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -3 $O/pytest_pp.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step augment timeout -k 10 300 python -u -m pytest tests/test_augment_gpu.py -x -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_aug.log 2>&1
tail -3 $O/pytest_aug.log
