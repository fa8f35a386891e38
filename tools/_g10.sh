cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fc1_dwconv" > gpurun_out/t_f.log 2>&1; rc=$?; tail -15 gpurun_out/t_f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-gemm gpurun_out/gemm_shapes.txt > gpurun_out/bench_extract.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
grep fc1dw gpurun_out/gemm_shapes.txt
SVK_FC1_DWCONV=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_extract_unfused.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract_unfused.log | cut -c1-330
