#!/bin/bash
# Round 6: PERM tiles' W-chunk swizzle by row bits (1, 3, 4) — bit-exactness vs the previous build, parity tests,
# same-box extraction and train A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z18
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step bxn timeout -k 10 300 python tools/perm_bitexact.py $O/pn.pt > $O/bxn.log 2>&1
SVK_LIB=$PWD/ab/libsvk_base.so step bxb timeout -k 10 300 python tools/perm_bitexact.py $O/pb.pt > $O/bxb.log 2>&1
step cmp python tools/perm_bitexact.py --compare $O/pn.pt $O/pb.pt > $O/cmp.log 2>&1
grep -c bit-identical $O/cmp.log
rm -f $O/pn.pt $O/pb.pt
step pytest timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py tests/test_train_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or headline or train_step" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for L in new base; do
  if [ $L = base ]; then export SVK_LIB=$PWD/ab/libsvk_base.so; else unset SVK_LIB; fi
  step x$L timeout -k 10 200 $B > $O/x_${L}_$i.log 2>&1
  echo "extract $L run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/x_${L}_$i.log | head -1)"
done; done
for i in 1 2; do for L in new base; do
  if [ $L = base ]; then export SVK_LIB=$PWD/ab/libsvk_base.so; else unset SVK_LIB; fi
  step t$L timeout -k 10 300 python bench.py --workload train --no-cpu-baseline --steps 40 --warmup 5 > $O/t_${L}_$i.log 2>&1
  echo "train $L run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/t_${L}_$i.log | head -1)"
done; done
