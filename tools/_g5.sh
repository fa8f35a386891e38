cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-gemm gpurun_out/gemm_shapes.txt > gpurun_out/bench_extract.log 2>&1; rc=$?; tail -1 gpurun_out/bench_extract.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_train.log 2>&1; rc=$?; tail -1 gpurun_out/bench_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_x.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_f.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_w.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t -o run -- python bench.py --workload train --no-graph --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_t.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmct_f -o run -- python bench.py --workload train --no-graph --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmct_f.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmct_w -o run -- python bench.py --workload train --no-graph --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmct_w.log 2>&1 || exit 1
echo done
