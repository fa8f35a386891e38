#!/bin/bash
# Round 5: gemm_pk SGPR-base DMA addressing — GEMM tests, sweep, headline parity, step bench, fc1 counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step gemmtests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or pingpong or persistent or conv" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gemm.log 2>&1
tail -1 $O/pytest_gemm.log
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step head timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_headline.log 2>&1
grep -E "passed|failed" $O/pytest_headline.log | tail -2
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
step bench1 timeout -k 10 200 $B > $O/bench1.log 2>&1; grep -o '"value": [0-9.]*' $O/bench1.log | head -1
step bench2 timeout -k 10 200 $B > $O/bench2.log 2>&1; grep -o '"value": [0-9.]*' $O/bench2.log | head -1
export SHAPE=50176,1280,320,0 ITERS=5
step pmc timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc -o run -- python tools/gemm_prof.py > $O/pmc.log 2>&1
