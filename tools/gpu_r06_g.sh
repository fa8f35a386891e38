#!/bin/bash
# Round 6: 192 x 128 gemm_pk tile (two workgroups per CU, 17 % fewer operand bytes per FLOP) vs the shipping tiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step sweep timeout -k 10 400 python tools/pk_cfg_sweep.py --cfgs=-1,88,100 > $O/sweep.txt 2>&1
grep -v amdgpu.ids $O/sweep.txt | cut -c1-250
