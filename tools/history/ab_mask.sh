#!/bin/bash
# A/B of the bs 32 group-analysis mask kernel's blocks per wave (lib_var/mask_nb{1,2,4,8}.so,
# -DSPMM_MASK32_NB): the group tests on one variant, then per variant the grouped bs 32 workloads
# under a rocprofv3 kernel trace (grp_mask32_kernel and the whole analysis). The release library
# is restored at the end. Output in gpurun_out/ab_mask/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
L=spmm-denseblock_amd/lib; O=$R/gpurun_out/ab_mask; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
restore() { cp $O/release.so $L/libspmm_hip.so; }
cp spmm-denseblock_amd/lib_var/mask_nb${TNB:-4}.so $L/libspmm_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsr.py -q -x --timeout 120 --timeout-method thread \
  -k "group or grouped or random_shapes_bits" > $O/pytest.log 2>&1; rc=$?
echo "tests nb${TNB:-4}: $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { restore; exit $rc; }
for rep in 1 2; do
for v in ${VS:-1 2 4 8}; do
  cp spmm-denseblock_amd/lib_var/mask_nb$v.so $L/libspmm_hip.so
  for w in reddit_bsr32_grp products_bsr32_grp; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${v}_${w}_$rep -o kt \
       --output-format csv -- python3 $R/bench.py --workload $w --steps 5 --warmup 2 \
       --no-cpu-baseline) > $O/${v}_${w}_$rep.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "nb$v $w rc=$rc"; restore; exit $rc; }
    an=$(grep '^{' $O/${v}_${w}_$rep.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r.get('analysis_ms'))")
    f=$(find $O/kt_${v}_${w}_$rep -name "*kernel_stats.csv" | head -1)
    mk=$(python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'grp_mask32' in r['Name'] or 'grp_fillc' in r['Name']: print(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1), end='  ')
")
    echo "nb$v $w rep$rep ms/analysis: $an | $mk"
  done
done
done
restore
