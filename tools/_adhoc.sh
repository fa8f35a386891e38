cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python bench.py --dtype bf16 --other-dtypes fp16 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/b_bf16first.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp16 --other-dtypes bf16 --no-cpu-baseline --steps 20 --warmup 40 > gpurun_out/b_fp16warm.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix -o run -- python bench.py --dtype fp16 --other-dtypes bf16 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_mix.log 2>&1
echo rc=$?
