#!/bin/bash
# Round 6: depthwise 3x3 variants with GELU + pre-activation store (the train forward's stages 3-4 form)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z2
mkdir -p $O
DW_ACT=gelu timeout -k 10 300 python tools/dw_train_bench.py > $O/dw_gelu.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/dw_gelu.txt; exit $rc
