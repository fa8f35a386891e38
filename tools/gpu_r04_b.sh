#!/bin/bash
# gemm_pp bring-up (parity tests, sweep vs hipBLASLt) + the round-4 first checks (hipBLASLt kernel names,
# train / temporal suites at HEAD, the new s2d / b3 tests).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pptest timeout -k 10 150 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "pingpong" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -3 $O/pytest_pp.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step blaslt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blaslt -o run -- python tools/blaslt_names.py > $O/blaslt.log 2>&1
step new timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py -q -rf -k "s2d or b3" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1
tail -3 $O/pytest_new.log
step train timeout -k 10 700 python -u -m pytest tests/test_train_gpu.py tests/test_temporal_train_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_train.log 2>&1
tail -3 $O/pytest_train.log
