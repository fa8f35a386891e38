cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prompt_ln or attn_block" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_pl.log 2>&1; rc=$?; tail -12 gpurun_out/t_pl.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_m.log 2>&1; rc=$?; tail -2 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do SVK_FUSED_PROMPT_LN=$v timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 30 --warmup 5 2>/dev/null | grep -o "\"value\": [0-9.]*" | sed "s/^/prompt_ln=$v /"; done
