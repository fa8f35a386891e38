#!/bin/bash
# split-K patchify conv row tiles (SVK_SPLITK_BM 64 / 128): parity, isolated conv timing, whole-step A/B;
# 128 x 160 tiles on the stage-3 q / proj shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
SVK_SPLITK_BM=128 step tests timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv2d_ln_sequence_reduction" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
step sweep timeout -k 10 300 python tools/pk_cfg_sweep.py --cfgs=-1,10,40 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log | head -4
for r in a b; do for v in 64 128; do
  SVK_SPLITK_BM=$v step bench$v$r timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 1500 --warmup 20 > $O/bench_$v$r.log 2>&1
  echo "bm=$v $(grep -o '"value": [0-9.]*' $O/bench_$v$r.log | head -1)"
done; done
for v in 64 128; do
  SVK_SPLITK_BM=$v step census$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census$v -o run -- python tools/graph_step_census.py run > $O/census$v.log 2>&1
  python tools/graph_step_census.py analyse $(find $O/census$v -name '*kernel_trace.csv' | head -1) --seq $O/seq$v.txt | tail -2 | cut -c1-100
  grep -E "PkCfgILi64ELi64|PkCfgILi128ELi64ELi2ELi2ELi2EEELb0ELb0ELi1ELb0ELb1|splitk" $O/seq$v.txt | awk '{s+=$2} END {print "split-K conv + LN per step:", s, "us"}'
done
