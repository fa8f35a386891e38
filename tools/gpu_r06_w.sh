#!/bin/bash
# Round 6: counters of the stage-3 flow cross-attention (attention_mfma_bf16_res<f16, 64, 4>)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
export ITERS=5
timeout -k 10 120 python tools/attn_fwd_prof.py > $O/warm.log 2>&1 || { tail -5 $O/warm.log; exit 1; }
run() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/attn_fwd_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA
run b SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU
run c TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
python tools/pmc_db.py attention_mfma $O/a/run_results.db $O/b/run_results.db $O/c/run_results.db
