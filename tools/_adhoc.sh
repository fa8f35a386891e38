cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mamba_gpu.py tests/test_temporal_train_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mb.log 2>&1; rc=$?; tail -2 gpurun_out/t_mb.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 400 python bench.py --workload tecno_train --temporal mamba --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_tt.log 2>&1; grep -o '"value": [0-9.]*' gpurun_out/b_tt.log | head -1; done
