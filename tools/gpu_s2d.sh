#!/bin/bash
# Stem space-to-depth round: parity (kernel, model goldens, B=256 headline, train), then a same-box
# interleaved extraction A/B of SVK_STEM_S2D.  Output under gpurun_out/s2d/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/s2d; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_models_gpu.py tests/test_headline_gpu.py tests/test_train_gpu.py -k "stem or gauss or models or headline or golden or prompt" \
  > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for e in SVK_STEM_S2D=0 SVK_STEM_S2D=1 SVK_STEM_S2D=0 SVK_STEM_S2D=1; do
  v=$(env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-dtypes none 2>>$O/ab.err \
      | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "extract $e: $v" | tee -a $O/ab.log
done
