#!/bin/bash
# A/B of the very shallow segment rule (SPMM_BSR_SEGF: segment waves per resident slot, 0 =
# off) on the reference sweep's bs 32 cells, with the TUNING library (lib_tuning/, copied over
# lib/ for the run, the release library restored at the end). Output in gpurun_out/ab_seg/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_seg; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so $L/libspmm_hip.so
for f in ${FS:-0 3 2 4 6}; do
  SPMM_BSR_SEGF=$f timeout -k 10 300 python -u tools/ref_sweep.py --densities ${PS:-0.02,0.002} \
    --bs ${BSS:-32} --dims ${DIMS:-64,128,256} --transB 0,1 --skip-csr --reps 10 \
    > $O/sweep_f$f.jsonl 2> $O/sweep_f$f.log; rc=$?
  echo "F=$f rc=$rc"
  python3 -c "
import json,sys
for l in open('$O/sweep_f$f.jsonl'):
    r=json.loads(l); print('F=$f', r.get('p'), r.get('bs'), r.get('dim'), r.get('transB'), r.get('ms'))"
  [ $rc -ne 0 ] && break
done
cp $O/release.so $L/libspmm_hip.so
