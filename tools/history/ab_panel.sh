#!/bin/bash
# A/B of the panel stream's stage depth (lib_var/d{22,32,43}.so: D at the 64- / 128-column tile)
# on the reference sweep's p = 2e-2 / 2e-3 bs 32 cells, transB = 1, two interleaved passes, after
# a bitwise test per variant. The release library is restored at the end. Output in
# gpurun_out/ab_panel/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_panel; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
restore() { cp $O/release.so $L/libspmm_hip.so; }
for v in ${VS:-d22 d32 d43}; do
  cp spmm-denseblock_amd/lib_var/$v.so $L/libspmm_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread \
    -k panel_stream > $O/pytest_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 $O/pytest_$v.log)"
  [ $rc -ne 0 ] && { restore; exit $rc; }
done
for rep in 1 2; do
for v in ${VS:-d22 d32 d43}; do
  cp spmm-denseblock_amd/lib_var/$v.so $L/libspmm_hip.so
  timeout -k 10 300 python -u tools/ref_sweep.py --densities 0.02,0.002 --bs 32 --dims 64,128,256 \
    --transB 1 --skip-csr --reps 10 > $O/sweep_${v}_$rep.jsonl 2> $O/sweep_${v}_$rep.log; rc=$?
  [ $rc -ne 0 ] && { restore; exit $rc; }
  python3 -c "
import json
print('$v', 'rep$rep', ' '.join(f\"{r['p']}/{r['dim']}:{r['ms']}\" for r in map(json.loads, open('$O/sweep_${v}_$rep.jsonl'))))"
done
done
restore
