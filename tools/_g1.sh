cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm or conv" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gemm_bench.py --reps 10 > gpurun_out/gemm_pk_tuning.txt 2>&1; rc=$?; cat gpurun_out/gemm_pk_tuning.txt | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-gemm gpurun_out/gemm_shapes.txt > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
