#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step dbg71 timeout -k 10 120 python -u tools/pp_debug.py 71 > $O/dbg71.log 2>&1
grep -v amdgpu.ids $O/dbg71.log
step pptest timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "pingpong" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -2 $O/pytest_pp.log
step square timeout -k 10 200 python -u tools/pp_square.py > $O/square.log 2>&1
grep -v amdgpu.ids $O/square.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
