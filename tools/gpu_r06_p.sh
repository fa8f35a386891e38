#!/bin/bash
# Round 6: depthwise 3x3 variants at the train step's data-gradient shapes (+ their parity tests)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "dwconv and not lds_variant" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
step bench timeout -k 10 300 python tools/dw_train_bench.py > $O/dw.txt 2>&1
grep -v amdgpu.ids $O/dw.txt
