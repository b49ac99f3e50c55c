#!/bin/bash
# A/B of column-range segments (SPMM_BSR_XSPLIT=R, TUNING library: every bs 32 block row cut
# into R block-column ranges, range r on XCD r % 8, partials summed in range order) on the
# reference sweep's bs 32 / 64 cells. First the tolerance test of long rows under R = 8 / 16.
# The release library is restored at the end. Output in gpurun_out/ab_xsplit/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_xsplit; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so $L/libspmm_hip.so
for r in 8 16; do
  SPMM_BSR_XSPLIT=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 \
    --timeout-method thread -k "long_rows_shallow or segments_with_staged" > $O/pytest_r$r.log 2>&1; rc=$?
  echo "R=$r tests: $(tail -1 $O/pytest_r$r.log)"
  [ $rc -ne 0 ] && { cp $O/release.so $L/libspmm_hip.so; exit $rc; }
done
for r in ${RS:-0 8 16 32}; do
  SPMM_BSR_XSPLIT=$r timeout -k 10 300 python -u tools/ref_sweep.py --densities ${PS:-0.02} \
    --bs ${BSS:-32} --dims ${DIMS:-64,128,256} --transB 0,1 --skip-csr --reps 10 \
    > $O/sweep_r$r.jsonl 2> $O/sweep_r$r.log; rc=$?
  python3 -c "
import json
for l in open('$O/sweep_r$r.jsonl'):
    r=json.loads(l); print('R=$r', r['p'], r['bs'], r['dim'], r['transB'], r['ms'])"
  [ $rc -ne 0 ] && break
done
cp $O/release.so $L/libspmm_hip.so
