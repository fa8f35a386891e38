#!/bin/bash
# Round 6: LayerNorm backward with four row groups per iteration — parity tests, same-box train A/B vs the previous build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z9
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
#step pytest timeout -k 10 900 python -u -m pytest tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "wgrad or train_step" > $O/pytest.log 2>&1
#tail -2
for i in 1 2; do for L in 512_512 1024_256 256_512 2048_128; do
  SVK_SKINNY_WG=${L%_*} SVK_SKINNY_MINROWS=${L#*_} step train$L timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/train_${L}_$i.log 2>&1
  echo "skinny wg_minrows $L run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/train_${L}_$i.log | head -1)"
done; done
