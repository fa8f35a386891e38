#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04dbg
timeout -k 10 200 python -u tools/aug_debug.py > gpurun_out/r04dbg/aug.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/r04dbg/aug.log
