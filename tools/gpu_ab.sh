#!/bin/bash
# Same-box interleaved A/B of the extraction bench over env settings: AB="VAR=a VAR=b ..." ROUNDS=n
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for k in $(seq ${ROUNDS:-3}); do
  for e in $AB; do
    v=$(env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none 2>/dev/null | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$e: $v"
  done
done
