#!/bin/bash
# Round 6: transposed-score attention-backward dQ kernel v2 (K / V staged in LDS) — parity tests + per-shape timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "attention_bwd" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
step bench timeout -k 10 300 python tools/attn_bwd_bench.py > $O/bench.txt 2>&1
grep -v amdgpu.ids $O/bench.txt
