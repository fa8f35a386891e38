cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dwconv" > gpurun_out/t_dw.log 2>&1; rc=$?; tail -2 gpurun_out/t_dw.log; [ $rc -eq 0 ] || exit $rc
SVK_DW_LDS=0 timeout -k 10 120 python tools/stencil_bench.py > gpurun_out/stencil_strip.txt 2>&1 || exit 1
timeout -k 10 120 python tools/stencil_bench.py > gpurun_out/stencil_lds.txt 2>&1 || exit 1
SVK_DW_LR=2 timeout -k 10 120 python tools/stencil_bench.py > gpurun_out/stencil_lds_r2.txt 2>&1 || exit 1
SVK_DW_LR=8 timeout -k 10 120 python tools/stencil_bench.py > gpurun_out/stencil_lds_r8.txt 2>&1 || exit 1
grep -h dwconv gpurun_out/stencil_*.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_extract.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_train.log 2>&1; rc=$?; tail -1 gpurun_out/bench_train.log
