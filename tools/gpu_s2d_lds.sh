#!/bin/bash
# Space-to-depth packing kernels (LDS-staged Gaussian, float4 frame/flow packing): parity, their rocprofv3
# kernel times inside the extraction step, and the bench line.  Output under gpurun_out/s2dlds/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/s2dlds; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
export SVK_S2D_PACK_VEC=1
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_models_gpu.py tests/test_headline_gpu.py -k "stem or gauss or models or headline or golden or prompt" -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --other-dtypes none --steps 10 --warmup 2 > $O/prof.log 2>&1
python tools/prof_stats.py $O/prof/run_kernel_stats.csv auto:mean_rows_kernel 45 > $O/stats.txt
grep -E "total|s2d|gauss" $O/stats.txt | cut -c1-150
for k in 0 1 0 1; do
  step bench env SVK_S2D_PACK_VEC=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none > $O/bench.log 2>&1
  echo "SVK_S2D_PACK_VEC=$k $(grep '^{' $O/bench.log | tail -1 | cut -c1-110)" | tee -a $O/ab.log
done
