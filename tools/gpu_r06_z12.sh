#!/bin/bash
# Round 6: where the flow encoder starts on the side stream (SVK_FLOW_AFTER_STAGE: -1 fork, 0 after stage 1, 1 after
# stage 2) — headline parity, same-box extraction-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z12
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
SVK_FLOW_AFTER_STAGE=0 step pytest timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "benched_config_fp16" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for v in -1 0 1; do
  SVK_FLOW_AFTER_STAGE=$v step b$v timeout -k 10 200 $B > $O/b_${v}_$i.log 2>&1
  echo "FLOW_AFTER_STAGE=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$i.log | head -1)"
done; done
