cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_sel.log 2>&1; rc=$?; tail -2 gpurun_out/t_sel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/precision_report.py 256 > gpurun_out/precision_b256.txt 2>&1 || exit $?
grep -E "^(fp16|bf16|fp32) B" gpurun_out/precision_b256.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b.log 2>&1; rc=$?; grep -o "\"value\": [0-9.]*" gpurun_out/b.log | head -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pk_cfg_sweep.py > gpurun_out/pk_sweep.log 2>&1; rc=$?; cat gpurun_out/pk_sweep.log | grep -v amdgpu.ids; exit $rc
