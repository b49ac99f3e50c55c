#!/bin/bash
# The group analysis on one GPU box: its GPU tests, then the grouped workloads' lines under a
# rocprofv3 kernel trace (the analysis kernels' durations: masks, grp_build PASS 1 / 2, the
# held masks, the fill) into gpurun_out/grp_$TAG/. A GPU fault, abort or time limit stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/grp_${TAG:-x}; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py -q -x --timeout 120 --timeout-method thread \
  -k "group or grouped" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; stop $rc
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
fi
for w in ${WLS:-reddit_bsr32_grp products_bsr32_grp products_bsr16_f16_grp}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$w -o kt --output-format csv \
     -- python3 $R/bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline) > $O/$w.log 2>&1
  rc=$?; stop $rc
  grep '^{' $O/$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', 'ms', r['ms_per_step'], 'analysis_ms', r.get('analysis_ms'))"
  f=$(find $O/kt_$w -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && python3 - "$f" <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("grp_build", "grp_wmask", "fill_kernel", "analysis_kernel", "grp_mask", "grp_stats", "scan_kernel")):
        print(f'  {int(r["Calls"]):4d} {float(r["AverageNs"]) / 1e3:9.1f} us  {n[:80]}')
EOF
done
exit 0
