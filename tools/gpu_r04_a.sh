#!/bin/bash
# Round-4 first GPU session: hipBLASLt kernel names on the MFMA-bound shapes (the yardstick the new
# GEMM is measured against), then the train / temporal GPU suites at HEAD (they were last
# run before the float4 s2d packing became the default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step blaslt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blaslt -o run -- python tools/blaslt_names.py > $O/blaslt.log 2>&1
cat $O/blaslt.log | grep -v amdgpu.ids
step train timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_temporal_train_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_train.log 2>&1
tail -3 $O/pytest_train.log
step new timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py -q -rf -k "s2d or b3" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1
tail -3 $O/pytest_new.log
