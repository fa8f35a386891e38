cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -k b88 -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider > gpurun_out/t_b88.log 2>&1; rc=$?; tail -2 gpurun_out/t_b88.log; grep "B=88" gpurun_out/t_b88.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
R=r02 bash tools/gpu_prof.sh
