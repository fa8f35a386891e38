cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "persistent or dwconv or conv2d or gemm" > gpurun_out/t_k.log 2>&1; rc=$?; tail -2 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune_bench.py all --rounds 5 --reps 5 > gpurun_out/tune.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/tune.txt; exit $rc
