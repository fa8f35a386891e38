#!/bin/bash
# One GPU session: kernel tests -> model tests -> smoke -> bench.  Stops at the first step that
# faults / aborts / times out (exit codes other than 0 = pass, 1 = test assertion failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -3 gpurun_out/pytest_kernels.log; ok $rc || exit $rc
[ "$rc" -eq 0 ] || exit 1
timeout -k 10 900 python -m pytest tests/test_models_gpu.py -m gpu -q > gpurun_out/pytest_models.log 2>&1
rc=$?; echo "models rc=$rc"; tail -3 gpurun_out/pytest_models.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
exit $rc
