#!/bin/bash
# Quick GPU session: full GPU test suite -> precision report at the benched batch -> extraction bench
# (fp16 headline + bf16 / fp32 extra keys).  Each GPU step has its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 240 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
grep -E "^(fp32|fp16|bf16) B=" $O/pytest_gpu.log | head
step precision timeout -k 10 300 python tools/precision_report.py 256 > $O/precision_b256.txt 2>&1
cat $O/precision_b256.txt | cut -c1-400
step bench_x timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 5 > $O/bench_extract.log 2>&1
tail -1 $O/bench_extract.log | cut -c1-1500
