#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step square timeout -k 10 200 python -u tools/pp_square.py > $O/square.log 2>&1
grep -v amdgpu.ids $O/square.log
step wgtest timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q -rf -k "test_conv_wgrad_dgrad or test_train_step_b88 or test_gemm_wgrad" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_train.log 2>&1
tail -3 $O/pytest_train.log
step train timeout -k 10 400 python bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --dump-gemm $O/train_gemm_shapes.txt > $O/bench_train.log 2>&1
grep '^{' $O/bench_train.log | cut -c1-300
grep -E "gemm_kernel|wgrad_kernel" $O/train_gemm_shapes.txt | head -30
