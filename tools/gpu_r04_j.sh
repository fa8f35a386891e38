#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "conv2d_s2d_ln or mixffn_rw or fc1dw" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_stem.log 2>&1; rc=$?
echo "stem tests rc=$rc"; tail -2 $O/pytest_stem.log; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "SVK_RW_VAR=2" "SVK_STEM_LN=0" "SVK_RW_VAR=2 SVK_STEM_LN=0"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_headline_gpu.py -q -rf -s -k "b3_fp16 or b2_fp16" --timeout 250 --timeout-method thread -p no:cacheprovider > $O/head.log 2>&1; rc=$?
  echo "[$v] rc=$rc"; grep -E "fp16 B=256|passed|failed" $O/head.log | head -4
  [ $rc -le 1 ] || exit $rc
done
for v in "X=0" "SVK_STEM_LN=0" "SVK_RW_VAR=2" "X=0" "SVK_STEM_LN=0" "SVK_RW_VAR=2"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-other-workloads --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
  echo "[$v] $(grep '^{' $O/bench.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python -u tools/conv_bench.py > $O/conv_bench.log 2>&1; echo "conv_bench rc=$?"
grep -v amdgpu.ids $O/conv_bench.log
