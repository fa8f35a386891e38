#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step dwtest timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "mixffn_dw_fc2" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_dw.log 2>&1
tail -2 $O/pytest_dw.log
step dwbench timeout -k 10 200 python -u tools/dwfc2_bench.py > $O/dwbench.log 2>&1
grep -v amdgpu.ids $O/dwbench.log
step models timeout -k 10 500 python -u -m pytest tests/test_headline_gpu.py tests/test_models_gpu.py -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_models.log 2>&1
tail -2 $O/pytest_models.log
step bench timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-other-workloads --no-cpu-baseline > $O/bench.log 2>&1
grep '^{' $O/bench.log | cut -c1-400
