cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_block" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ab.log 2>&1; rc=$?; tail -15 gpurun_out/t_ab.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_m.log 2>&1; rc=$?; tail -2 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/precision_report.py 256 > gpurun_out/precision_b256.txt 2>&1; grep -E "^(fp16|bf16|fp32) B" gpurun_out/precision_b256.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b.log 2>&1; rc=$?; grep -o '"value": [0-9.]*' gpurun_out/b.log; exit $rc
