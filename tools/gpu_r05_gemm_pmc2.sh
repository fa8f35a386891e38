#!/bin/bash
# Round 5: SQ / TCC counters of the dominant gemm_pk shapes after the scalar-base DMA addressing
# (stage-3 fc1 and the head's decode-fuse GEMM), each pass its own run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g2
mkdir -p $O
rung() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o run -- python tools/gemm_prof.py > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }; echo "pass $n ok"; }
for sh in "50176,1280,320,0" "12544,2048,1024,0"; do
  export SHAPE=$sh
  t=$(echo $sh | tr ',' '_')
  rung ${t}_a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS
  rung ${t}_b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM
  rung ${t}_c TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
done
