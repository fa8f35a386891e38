#!/bin/bash
# dw_fc2_mx counter passes (one rocprofv3 --pmc run per pass), for SVK_DWFC2_DIAG in $DIAGS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/dwfc2_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
for d in ${DIAGS:-0}; do
  export SVK_DWFC2_DIAG=$d
  run a$d SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS
  run b$d SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC
  run c$d SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_EXP
done
