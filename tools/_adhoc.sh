cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_headline_gpu.py tests/test_train_gpu.py -x -q --timeout 380 --timeout-method thread -p no:cacheprovider > gpurun_out/t_g.log 2>&1; rc=$?; tail -2 gpurun_out/t_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/precision_report.py 256 > gpurun_out/precision_b256.txt 2>&1; grep -E "B=256" gpurun_out/precision_b256.txt | head -4
