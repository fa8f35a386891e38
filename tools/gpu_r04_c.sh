#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
timeout -k 10 200 python -u -m pytest tests/test_augment_gpu.py tests/test_preproc_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_aug.log 2>&1; echo aug rc=$?
tail -2 $O/pytest_aug.log
step pptest timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k "pingpong" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pp.log 2>&1
tail -3 $O/pytest_pp.log
step sweep timeout -k 10 300 python -u tools/pk_cfg_sweep.py --reps 30 > $O/sweep.log 2>&1
grep -v amdgpu.ids $O/sweep.log
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run > $O/census.log 2>&1
python tools/graph_step_census.py analyse $(find $O/census -name '*kernel_trace.csv' | head -1) > $O/census.txt; cat $O/census.txt
