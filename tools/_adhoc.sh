cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mamba_gpu.py tests/test_kernels_gpu.py -k "mamba or ragged or gemm or conv" -x -q --timeout 240 --timeout-method thread > gpurun_out/t_k.log 2>&1; rc=$?; tail -3 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mamba --steps 5 --warmup 2 --cpu-baseline-seconds 10 > gpurun_out/b_mamba.log 2>&1; rc=$?; grep '^{' gpurun_out/b_mamba.log | cut -c1-1200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b.log 2>&1; rc=$?; grep -o '"value": [0-9.]*' gpurun_out/b.log; exit $rc
