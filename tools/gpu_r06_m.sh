#!/bin/bash
# Round 6: attention backward per shape (transposed-score vs round-5 dQ kernel), counters of the 196-key dQ launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python tools/attn_bwd_bench.py > $O/bench.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.txt; [ $rc -eq 0 ] || exit $rc
P="python tools/attn_bwd_bench.py --only 4 --reps 3 --rounds 1 --variants"
run() { local n=$1 v=$2; shift 2; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- $P $v > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
for v in 1 0; do
  run a$v $v SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS
  run b$v $v SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT
  run c$v $v TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
  python tools/pmc_db.py attn_bwd_dq $O/a$v/run_results.db $O/b$v/run_results.db $O/c$v/run_results.db
done
