#!/bin/bash
# GEMM tile sweep (every pk_cfg variant + hipBLASLt, interleaved in one process) + the LFB pipeline test
# + the PCIe-inclusive lfb bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u tools/pk_cfg_sweep.py --reps 30 > $O/pk_sweep.log 2>&1; rc=$?
cat $O/pk_sweep.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k "lfb" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_lfb.log 2>&1; rc=$?
tail -n 5 $O/pytest_lfb.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload lfb --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_lfb.log 2>&1 || exit 1
tail -n 1 $O/bench_lfb.log | cut -c1-600
