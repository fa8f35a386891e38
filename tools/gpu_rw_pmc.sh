#!/bin/bash
# PMC passes over the mixffn_rw kernel alone (tools/mixffn_bench.py --only rw); counter list first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/rwpmc; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1; echo "list rc=$?"
grep -oE "SQ_[A-Z_0-9]+" $O/avail.txt | sort -u > $O/sq_names.txt; wc -l < $O/sq_names.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1)); ok=1
  for c in $P; do grep -qx "$c" $O/sq_names.txt || { echo "missing $c"; ok=0; }; done
  [ $ok -eq 1 ] || continue
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/p$n -o p$n --output-format csv -- python3 tools/mixffn_bench.py --only rw --reps 3 > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -3 $O/p$n.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
