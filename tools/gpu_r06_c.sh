#!/bin/bash
# Round 6: GELU on packed f32 pairs (mixffn_rwd, fc1dw_rw, dw_fc2_mx): parity tests, per-kernel A/B, interleaved
# whole-step A/B; current gemm_pp / gemm_wt status on the big shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
[ -n "$SKIP_PYTEST" ] || step pytest timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_gpu.py tests/test_models_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "mixffn or dw_fc2 or b3 or benched or golden or fc1" > $O/pytest.log 2>&1
tail -2 $O/pytest.log; grep -h "b3\|max" $O/pytest.log | head -5
for i in 1 2; do for v in 0 1; do
  SVK_GELU_PK=$v step kab$v timeout -k 10 120 python tools/gelu_pk_ab.py > $O/kab_${v}_$i.txt 2>&1; grep SVK $O/kab_${v}_$i.txt | cut -c1-300
done; done
for i in 1 2 3; do for v in 0 1; do
  SVK_GELU_PK=$v step bench$v timeout -k 10 200 python bench.py --no-other-workloads --no-cpu-baseline --other-dtypes none --steps 200 --warmup 20 > $O/bench_${v}_$i.log 2>&1
  echo "GELU_PK=$v run $i: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.log | head -1)"
done; done
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,70,71,90,92,100 --shapes "s3 fc1,head,s4 fc1,s3 fc2" > $O/sweep.txt 2>&1
grep -v amdgpu.ids $O/sweep.txt | sed 's/ d=0.0e+00//g' | cut -c1-330
