cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention or mstcn" -x -q --timeout 240 --timeout-method thread > gpurun_out/t_k.log 2>&1; rc=$?; tail -3 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_m.log 2>&1; rc=$?; tail -3 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mstcn --steps 5 --warmup 2 --cpu-baseline-seconds 10 > gpurun_out/b_mstcn.log 2>&1; rc=$?; grep '^{' gpurun_out/b_mstcn.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b.log 2>&1; rc=$?; grep -o '"value": [0-9.]*' gpurun_out/b.log; grep -o '"other_dtypes".*' gpurun_out/b.log; exit $rc
