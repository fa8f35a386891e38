#!/bin/bash
# Per-stage prompt events (SVK_PROMPT_STAGE_EVENTS): model / headline parity, census of the step start, same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step tests timeout -k 10 500 python -u -m pytest tests/test_models_gpu.py tests/test_headline_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
step census timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/census -o run -- python tools/graph_step_census.py run > $O/census.log 2>&1
python tools/graph_step_census.py analyse $(find $O/census -name '*kernel_trace.csv' | head -1) --seq $O/seq.txt | tail -2 | cut -c1-90
for r in a b; do for v in 0 1; do
  SVK_PROMPT_STAGE_EVENTS=$v step bench$v$r timeout -k 10 200 python bench.py --no-cpu-baseline --other-dtypes none --no-other-workloads --steps 1500 --warmup 20 > $O/bench_$v$r.log 2>&1
  echo "stage_events=$v $(grep -o '"value": [0-9.]*' $O/bench_$v$r.log | head -1)"
done; done
