#!/bin/bash
# Round 6: stage-3 dwfc2_rw (f16, B = 256) counters — L2 request volume vs time (is the operand stream the bound?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
export ITERS=5
timeout -k 10 120 python tools/dwfc2_prof.py > $O/warm.log 2>&1 || { tail -5 $O/warm.log; exit 1; }
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/dwfc2_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
run a TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
run b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS
run c SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM
python tools/pmc_db.py dwfc2_rw $O/a/run_results.db $O/b/run_results.db $O/c/run_results.db
