#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
T="tests/test_train_gpu.py::test_train_step_grads_fp32_vs_oracle tests/test_train_gpu.py::test_train_ddp_rccl_world1_capture_replay tests/test_models_gpu.py::test_mstcn_ragged_videos_vs_per_video_and_oracle"
for v in "X=0" "SVK_NO_F32_SMALLM=1" "SVK_FLAT_ALIGN=0" "SVK_NO_WGRAD_PK_CONV=1"; do
  env $v timeout -k 10 400 python -u -m pytest $T -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?
  echo "[$v] rc=$rc $(tail -1 $O/t.log)"; grep -E "^FAILED" $O/t.log | head -6
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -q -rf -k "mixffn_rw or fc1dw or gemm_f32_smallm" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t2.log 2>&1; echo "kern rc=$? $(tail -1 $O/t2.log)"
