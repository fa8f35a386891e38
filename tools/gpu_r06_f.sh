#!/bin/bash
# Round 6: gemm_pk staged-epilogue stores with the non-temporal hint (SVK_PK_NT=1) vs default: per-shape sweep
# and interleaved whole-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
for v in 0 1; do
  SVK_PK_NT=$v step sweep$v timeout -k 10 200 python tools/pk_cfg_sweep.py --cfgs=-1 --rounds 3 --shapes "s3 fc1,s3 fc2,head,s4 fc1,s4 fc2,s2 fc2,s4 kv,s3 q/proj" > $O/sweep_$v.txt 2>&1
  echo "NT=$v"; grep -v amdgpu.ids $O/sweep_$v.txt | sed 's/ d=0.0e+00//g' | cut -c1-80
done
for i in 1 2 3; do for v in 0 1; do
  SVK_PK_NT=$v step bench$v timeout -k 10 200 python bench.py --no-other-workloads --no-cpu-baseline --other-dtypes none --steps 200 --warmup 20 > $O/bench_${v}_$i.log 2>&1
  echo "PK_NT=$v run $i: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.log | head -1)"
done; done
