#!/bin/bash
# Clock / power while the graph-replayed extraction step runs, library GEMM policy off / on (same box):
# is the whole step power-limited (DVFS), so that faster high-power GEMMs slow every other kernel?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
timeout -k 5 20 rocm-smi --showclocks --showpower > $O/smi_idle.txt 2>&1
for v in 0 1 0 1; do
  ( for i in $(seq 1 60); do timeout -k 2 5 rocm-smi --showclocks --showpower --csv 2>/dev/null | grep -v '^$'; sleep 0.25; done ) > $O/smi_lib$v.$RANDOM.csv &
  SP=$!
  SVK_LIBGEMM=$v step bench$v timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 1500 --warmup 20 > $O/bench_lib$v.log 2>&1
  kill $SP 2>/dev/null; wait $SP 2>/dev/null
  echo "lib=$v $(grep '^{' $O/bench_lib$v.log | cut -c90-200)"
done
