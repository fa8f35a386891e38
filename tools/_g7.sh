cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or bf16" > gpurun_out/t_a.log 2>&1; rc=$?; tail -3 gpurun_out/t_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_extract.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_x.log 2>&1 || exit 1
python tools/prof_stats.py gpurun_out/prof_x/run_kernel_stats.csv 7 12
