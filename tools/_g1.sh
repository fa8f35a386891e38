cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_train.log 2>&1; rc=$?; tail -1 gpurun_out/bench_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proft -o run -- python bench.py --workload train --no-graph --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1 || exit 1
