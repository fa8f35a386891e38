#!/bin/bash
# Iteration session: MixFFN ablations, persistent-GEMM stress, GPU suite (no -x), train + extraction benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 python -u tools/mixffn_bench.py --reps 20 > $O/mixffn_bench.log 2>&1 || exit 1
grep -v amdgpu.ids $O/mixffn_bench.log
timeout -k 10 240 python -u tools/pk_stress.py 10 > $O/pk_stress.log 2>&1 || exit 1
echo "pk_stress: $(grep -c 'unstable 0/10 (max 0)' $O/pk_stress.log) stable of $(grep -c unstable $O/pk_stress.log); bad: $(grep -c 'bad elems [1-9]' $O/pk_stress.log)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 6 $O/pytest_gpu.log | cut -c1-300
[ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || exit $rc
grep -E "^(config5|train_evp loop|RCCL|fp16 B=)" $O/pytest_gpu.log | head
timeout -k 10 400 python bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline --dump-gemm $O/train_gemm_shapes.txt > $O/bench_train.log 2>&1 || exit 1
tail -n 1 $O/bench_train.log | cut -c1-300
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none > $O/bench.log 2>&1 || exit 1
tail -n 1 $O/bench.log | cut -c1-300
