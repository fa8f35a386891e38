#!/bin/bash
# Library-GEMM shape subsets vs the clock: bench + sclk / power samples per SVK_LIBGEMM_MASK (same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
run() {  # $1 = tag, env already set by the caller
  ( for i in $(seq 1 50); do timeout -k 2 5 rocm-smi --showclocks --showpower --csv 2>/dev/null | grep card0; sleep 0.25; done ) > $O/smi_$1.csv &
  local SP=$!
  step bench_$1 timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --steps 1500 --warmup 20 > $O/bench_$1.log 2>&1
  kill $SP 2>/dev/null; wait $SP 2>/dev/null
  echo "$1 $(grep '^{' $O/bench_$1.log | cut -c120-175) sclk/W: $(awk -F, '{print $6"/"$10}' $O/smi_$1.csv | tr -d '()Mhz' | sort -t/ -k2 -n | tail -12 | head -8 | tr '\n' ' ')"
}
for r in a b; do
  SVK_LIBGEMM=0 run off$r
  SVK_LIBGEMM=1 SVK_LIBGEMM_MASK=1 run m1$r
  SVK_LIBGEMM=1 SVK_LIBGEMM_MASK=29 run m29$r
  SVK_LIBGEMM=1 SVK_LIBGEMM_MASK=12 run m12$r
done
