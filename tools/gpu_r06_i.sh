#!/bin/bash
# Round 6: stage-1 mixffn_rwd counters after the packed GELU (compare profiles/r05/mixffn_rwd_pmc.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 120 python tools/mixffn_prof.py 2>&1 | grep -v amdgpu.ids || exit 1
export ITERS=5
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/mixffn_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS
run b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC
run c SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM
python tools/pmc_summary.py mixffn_rwd $(find $O -name '*counter_collection.csv') > $O/summary.txt 2>&1; cat $O/summary.txt
