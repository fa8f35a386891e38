#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step dbg70 timeout -k 10 120 python -u tools/pp_debug.py 70 > $O/dbg70.log 2>&1
grep -v amdgpu.ids $O/dbg70.log
step dbg71 timeout -k 10 120 python -u tools/pp_debug.py 71 > $O/dbg71.log 2>&1
grep -v amdgpu.ids $O/dbg71.log
step pptest timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q -rf -k "(pingpong and not 72) or test_conv_wgrad_dgrad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -3 $O/pytest_pp.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 --no-sk > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step dbg72 timeout -k 10 120 python -u tools/pp_debug.py 72 > $O/dbg72.log 2>&1
grep -v amdgpu.ids $O/dbg72.log
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run > $O/census.log 2>&1
python tools/graph_step_census.py analyse $(find $O/census -name '*kernel_trace.csv' | head -1) > $O/census.txt; cat $O/census.txt
step train timeout -k 10 400 python bench.py --workload train --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --dump-gemm $O/train_gemm_shapes.txt > $O/bench_train.log 2>&1
grep -E "gemm_kernel|wgrad_kernel" $O/train_gemm_shapes.txt | head -40
