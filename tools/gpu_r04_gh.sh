#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04gh
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step dbg70 timeout -k 10 120 python -u tools/pp_debug.py 70 > $O/dbg70.log 2>&1
grep -v amdgpu.ids $O/dbg70.log | grep -c "bad 0/"
step pptest timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "pingpong" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -2 $O/pytest_pp.log
step square timeout -k 10 200 python -u tools/pp_square.py > $O/square.log 2>&1
grep -v amdgpu.ids $O/square.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step dwtest timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q -rf -k "mixffn or fc1dw or gemm_f32_smallm or test_gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_dw.log 2>&1
tail -2 $O/pytest_dw.log
step dwbench timeout -k 10 200 python -u tools/dwfc2_bench.py > $O/dwbench.log 2>&1
grep -v amdgpu.ids $O/dwbench.log
step models timeout -k 10 500 python -u -m pytest tests/test_headline_gpu.py tests/test_models_gpu.py -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_models.log 2>&1
tail -2 $O/pytest_models.log
step bench timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-other-workloads --no-cpu-baseline > $O/bench.log 2>&1
grep '^{' $O/bench.log | cut -c1-400
step train timeout -k 10 400 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline --no-other-workloads --dump-gemm $O/train_gemm_shapes.txt > $O/bench_train.log 2>&1
grep '^{' $O/bench_train.log | cut -c1-300
head -30 $O/train_gemm_shapes.txt
