cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_block" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ab.log 2>&1; rc=$?; tail -12 gpurun_out/t_ab.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_m.log 2>&1; rc=$?; tail -2 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_block_bench.py 2>&1 | grep -v amdgpu
for v in 0 1 0 1; do SVK_FUSED_ATTN_BLOCK=$v timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 30 --warmup 5 2>/dev/null | grep -o "\"value\": [0-9.]*" | sed "s/^/fused=$v /"; done
