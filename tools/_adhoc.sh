cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_headline_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; echo pytest=$?; tail -2 gpurun_out/pt.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b_graph.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-graph > gpurun_out/b_nograph.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype bf16 --other-dtypes fp16 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b_bf16.log 2>&1
echo rc=$?
