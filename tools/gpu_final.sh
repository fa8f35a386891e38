#!/bin/bash
# Round-end GPU session: full GPU suite -> smoke -> extraction profiles + PMC + bench (tools/gpu_prof.sh)
# -> train / temporal bench lines with CPU baselines.  Everything lands in gpurun_out/profiles_r02.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O/profiles_r02
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 380 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
R=r02 bash tools/gpu_prof.sh || exit $?
step bench_t timeout -k 10 300 python bench.py --workload train --steps 10 --warmup 3 --cpu-baseline-seconds 15 > $O/bench_train.log 2>&1
grep '^{' $O/bench_train.log > $O/profiles_r02/bench_train.jsonl
step bench_ms timeout -k 10 300 python bench.py --workload mstcn --steps 5 --warmup 2 --cpu-baseline-seconds 10 > $O/bench_mstcn.log 2>&1
grep '^{' $O/bench_mstcn.log > $O/profiles_r02/bench_mstcn_ragged.jsonl
step bench_mb timeout -k 10 300 python bench.py --workload mamba --steps 5 --warmup 2 --cpu-baseline-seconds 10 > $O/bench_mamba.log 2>&1
grep '^{' $O/bench_mamba.log > $O/profiles_r02/bench_mamba_ragged.jsonl
for f in $O/profiles_r02/bench_*; do echo "$f: $(grep -o '"value": [0-9.]*' $f | head -1)"; done
