#!/bin/bash
# A/B (TUNING library) of deeper A rings on the bs 32 column stream: SPMM_BSR_VARIANT 4418 / 4419
# / 4420 = NA 4 (three blocks ahead) at P 6 / 4 / 8 items in flight, against the shipped NA 3,
# P 6 (4416). Output in gpurun_out/ab_na4/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_na4; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so $L/libspmm_hip.so
SPMM_BSR_VARIANT=4418 timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 \
  --timeout-method thread -k "random_shapes_bits or long_rows or segments" > $O/pytest.log 2>&1; rc=$?
echo "tests: $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { cp $O/release.so $L/libspmm_hip.so; exit $rc; }
for rep in 1 2; do
for v in 4416 4418 4419 4420; do
  for w in products_bsr32 reddit_bsr32; do
    SPMM_BSR_VARIANT=$v timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 \
      --no-cpu-baseline --no-analysed-side > $O/bw_${v}_${w}_$rep.log 2>&1; rc=$?
    grep "^{" $O/bw_${v}_${w}_$rep.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$v', '$w', r['ms_per_step'], f.get('kernel_ms'), f.get('mfma_frac'))"
    [ $rc -ne 0 ] && { cp $O/release.so $L/libspmm_hip.so; exit $rc; }
  done
done
done
cp $O/release.so $L/libspmm_hip.so
