cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "conv2d_ln or persistent" > gpurun_out/t_k.log 2>&1; rc=$?; tail -3 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-gemm gpurun_out/gemm_shapes.txt > gpurun_out/bench_extract.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
grep -i "conv" gpurun_out/gemm_shapes.txt | head
