#!/bin/bash
# Round 6: deep-ring gemm_pk candidates (one 8-wave workgroup per CU, 3-4 K-steps of LDS-DMA in flight) vs the
# shipping 2-workgroup 128x128 tile, interleaved sweep on the MiT-b2 shapes + correctness of the new variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit $rc; }
step sweep timeout -k 10 400 python tools/pk_cfg_sweep.py --cfgs=-1,85,86,87,100 --shapes "s3 fc1,s3 fc2,head,s4 fc2,s4 fc1,s2 fc2,s4 kv" > $O/sweep.txt 2>&1
grep -v amdgpu.ids $O/sweep.txt | sed 's/ d=0.0e+00//g' | cut -c1-330
