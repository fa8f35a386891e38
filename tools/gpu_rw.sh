#!/bin/bash
# MixFFN register-window iteration: its parity tests, the MixFFN bench, then the GPU suite and the
# extraction bench.  A step that faults, aborts or times out ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "mixffn" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_rw.log 2>&1
rc=$?; echo "pytest rw rc=$rc"; tail -n 15 $O/pytest_rw.log | cut -c1-300
[ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || exit $rc
timeout -k 10 240 python -u tools/mixffn_bench.py --reps 20 > $O/mixffn_bench.log 2>&1 || exit 1
grep -v amdgpu.ids $O/mixffn_bench.log
[ "$rc" -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none --dump-gemm $O/gemm_shapes.txt > $O/bench.log 2>&1 || exit 1
tail -n 1 $O/bench.log | cut -c1-400
head -5 $O/gemm_shapes.txt
if [ -n "$FULL" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 $O/pytest_gpu.log | cut -c1-300
fi
