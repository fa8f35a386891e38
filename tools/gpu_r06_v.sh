#!/bin/bash
# Round 6: resident-K/V attention with its K / V staging loads issued before the LDS writes and Q one tile ahead —
# parity tests, kernel and extraction-step A/B against the previous build (ab/libsvk_base.so via SVK_LIB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py tests/test_models_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "attention or headline or b2 or b3" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for L in new base; do
  if [ $L = base ]; then export SVK_LIB=$PWD/ab/libsvk_base.so; else unset SVK_LIB; fi
  step kb$L timeout -k 10 200 python tools/attn_fwd_bench.py > $O/kb_$L.log 2>&1
  echo "$L: $(grep -v amdgpu $O/kb_$L.log | tr '\n' ' ')"
done
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for L in new base; do
  if [ $L = base ]; then export SVK_LIB=$PWD/ab/libsvk_base.so; else unset SVK_LIB; fi
  step bench$L timeout -k 10 200 $B > $O/bench_${L}_$i.log 2>&1
  echo "$L run $i: $(grep -o '"value": [0-9.]*' $O/bench_${L}_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${L}_$i.log | head -1)"
done; done
