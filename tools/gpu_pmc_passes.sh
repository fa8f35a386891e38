#!/bin/bash
# PMC passes (one rocprofv3 run each, counters per pass from PASS1..PASS4) over CMD; summaries per kernel
# substring KSUB via tools/pmc_summary.py.  Usage: PASS1="..." PASS2="..." CMD="python3 ..." KSUB=... bash this
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_${TAG:-x}; mkdir -p $O
n=0
for P in "$PASS1" "$PASS2" "$PASS3" "$PASS4"; do
  n=$((n+1)); [ -n "$P" ] || continue
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$n -o p$n --output-format csv -- $CMD > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -3 $O/p$n.log; exit 1; }
done
python3 tools/pmc_summary.py "$KSUB" $(find $O -name "*counter_collection.csv")
