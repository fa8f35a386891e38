#!/bin/bash
# gemm_pk epilogue diagnosis: run-to-run stability of every tile config (tools/pk_stress.py) for
#   v1 = the shipped library (no packed-FP32 VALU ops), v2 = packed-FP32 ops on, epilogue operands by
#   inline-asm loads (round-2 design), v3 = packed-FP32 ops on, compiler-visible epilogue loads;
# then a same-box interleaved extraction A/B of the three.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 python -u tools/pk_stress.py ${REPS:-10} > $O/pk_v1.log 2>&1 && echo v1 done &&
SVK_LIB=diag_libs/libsvk_v2.so timeout -k 10 240 python -u tools/pk_stress.py ${REPS:-10} > $O/pk_v2.log 2>&1 && echo v2 done &&
SVK_LIB=diag_libs/libsvk_v3.so timeout -k 10 240 python -u tools/pk_stress.py ${REPS:-10} > $O/pk_v3.log 2>&1 && echo v3 done &&
timeout -k 10 300 python -u -m pytest tests/test_temporal_train_gpu.py -k two_forwards -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/two_fwd.log 2>&1 && echo twofwd done || exit 1
for r in 1 2; do
  for v in v1 v2 v3; do
    if [ $v = v1 ]; then unset SVK_LIB; else export SVK_LIB=diag_libs/libsvk_$v.so; fi
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --other-dtypes none > $O/ab_$v.$r.log 2>&1 || exit 1
    echo "$v r$r $(tail -1 $O/ab_$v.$r.log | cut -c1-120)"
  done
done
