#!/bin/bash
# A/B of lib_var/*.so on the bs 32 column-stream workloads: per variant a few bs 32 tests, then
# the drop-in bench lines (no side entries). Restores the release library at the end.
# Output in gpurun_out/ab_cs2/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_cs2; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
for v in ${VARS:-$(ls spmm-denseblock_amd/lib_var | sed 's/\.so$//')}; do
  cp spmm-denseblock_amd/lib_var/$v.so $L/libspmm_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -q -x --timeout 120 --timeout-method thread -k "${TK:-segments or narrow or bsrmm_grouped_f32}" > $O/pytest_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 $O/pytest_$v.log)"
  [ $rc -ge 124 ] && { cp $O/release.so $L/libspmm_hip.so; exit $rc; }
  for w in ${WLS:-reddit_bsr32 reddit_rcm_bsr32 products_bsr32}; do
    timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-analysed-side > $O/bw_${v}_$w.log 2>&1; rc=$?
    grep "^{" $O/bw_${v}_$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$v', '$w', r['ms_per_step'], f.get('kernel_ms'), f.get('mfma_frac'))"
    [ $rc -ge 124 ] && { cp $O/release.so $L/libspmm_hip.so; exit $rc; }
  done
done
cp $O/release.so $L/libspmm_hip.so
