#!/bin/bash
# Round 6: PERM for the plain residual epilogue too (SVK_PK_PERM=2) — bit-exactness vs 1, parity, extraction A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z15
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
SVK_PK_PERM=2 step bx1 timeout -k 10 300 python tools/perm_bitexact.py $O/p1.pt > $O/bx1.log 2>&1
SVK_PK_PERM=1 step bx0 timeout -k 10 300 python tools/perm_bitexact.py $O/p0.pt > $O/bx0.log 2>&1
tail -1 $O/bx1.log | cut -c1-600
step cmp python tools/perm_bitexact.py --compare $O/p1.pt $O/p0.pt
rm -f $O/p1.pt $O/p0.pt
step pytest timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py tests/test_models_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or headline or b2 or b3" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
B="python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 200 --warmup 20"
for i in 1 2 3; do for v in 2 1; do
  SVK_PK_PERM=$v step b$v timeout -k 10 200 $B > $O/b_${v}_$i.log 2>&1
  echo "PK_PERM=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$i.log | head -1)"
done; done
