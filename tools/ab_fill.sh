#!/bin/bash
# A/B of lib_var/*.so on the group analysis (kernel trace of the grouped workloads per variant,
# tools/grp_analysis.sh without its tests). Restores the release library at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; mkdir -p gpurun_out
cp $L/libspmm_hip.so gpurun_out/release.so
for v in ${VARS:-$(ls spmm-denseblock_amd/lib_var | sed 's/\.so$//')}; do
  cp spmm-denseblock_amd/lib_var/$v.so $L/libspmm_hip.so
  echo "== $v"
  TESTS=0 TAG=$v bash tools/grp_analysis.sh; rc=$?
  [ $rc -ge 124 ] && { cp gpurun_out/release.so $L/libspmm_hip.so; exit $rc; }
done
cp gpurun_out/release.so $L/libspmm_hip.so
