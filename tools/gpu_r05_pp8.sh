#!/bin/bash
# Round 5: the parameter refresh 8 elements per thread (svk_pack_params8, SVK_PACK_PARAMS8): train + temporal
# train parity, the train-step A/B interleaved on one box; then mixffn_rwd's SQ counters (VALU-bound check)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05p8
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_temporal_train_gpu.py > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -60 $O/pytest_train.log; exit 1; }
echo "train: $(tail -1 $O/pytest_train.log)"
B="python bench.py --workload train --no-cpu-baseline --steps 20 --warmup 3"
for rep in 1 2; do
  for v in 1 0; do
    SVK_PACK_PARAMS8=$v timeout -k 10 300 $B > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.log; exit 1; }
    echo "pack8=$v: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
  done
done
export ITERS=5
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/mixffn_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS
run b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC
run c SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM
