#!/bin/bash
# dwconv XCD grouping (correctness, timing, FETCH/WRITE calibration), library-GEMM sweep, then the
# extraction FETCH pass alone with a longer limit (it was killed at 150 s in the closing session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step tests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q -k "dwconv or gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for x in 0 1 0 1; do SVK_DW_XCD=$x step dwt$x timeout -k 10 120 python tools/dw_calib.py 20 >> $O/dw_time.log 2>&1; done
cat $O/dw_time.log | grep xcd
for x in 0 1; do
  SVK_DW_XCD=$x step pmcf$x timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/dwf$x -o run -- python tools/dw_calib.py 3 > $O/dwf$x.log 2>&1
  SVK_DW_XCD=$x step pmcw$x timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/dww$x -o run -- python tools/dw_calib.py 3 > $O/dww$x.log 2>&1
done
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,60,71,80 > $O/sweep.log 2>&1
cat $O/sweep.log | grep -v amdgpu.ids
SVK_LIBGEMM=1 step sweep_pol timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1 > $O/sweep_pol.log 2>&1
cat $O/sweep_pol.log | grep -v amdgpu.ids
for v in 0 1 0 1; do SVK_LIBGEMM=$v step bench$v timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 20 --warmup 5 > $O/bench_lib$v.log 2>&1; echo "lib=$v $(grep '^{' $O/bench_lib$v.log | cut -c1-120)"; done
for v in 0 1; do SVK_DW_XCD=$v step benchx$v timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 20 --warmup 5 > $O/bench_x$v.log 2>&1; echo "xcd=$v $(grep '^{' $O/bench_x$v.log | cut -c1-120)"; done
step pmc_f timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python bench.py --no-cpu-baseline --other-dtypes none --no-graph --steps 1 --warmup 1 > $O/pmc_f.log 2>&1
