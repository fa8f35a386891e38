cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dwconv" > gpurun_out/t_dw.log 2>&1; rc=$?; tail -3 gpurun_out/t_dw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tune_bench.py dw --rounds 5 --reps 5 > gpurun_out/tune_dw.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/tune_dw.txt; exit $rc
