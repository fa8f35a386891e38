#!/bin/bash
# Round 6: tile sweep over the train step's extended-epilogue GEMMs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 500 python tools/ext_sweep.py > $O/ext_sweep2.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ext_sweep2.txt; exit $rc
