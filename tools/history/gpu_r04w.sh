#!/bin/bash
# Batched A-fragment fills of the group analysis and batched bs 16 analysis blocks:
# grouped and analysed tests, the four grouped workload lines (analysis_ms), a kernel
# trace of the bs 16 one, determinism. OUT names the output directory (default r04w).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-r04w}; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -m gpu -k "group or analys or f16" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; stop $rc
[ $rc -eq 0 ] || exit $rc
: > $O/workloads.jsonl
for w in reddit_bsr32_grp products_bsr32_grp products_bsr16_f16_grp products_rcm_bsr16_f16_grp; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw.log 2>&1; rc=$?; stop $rc
  grep '^{' $O/bw.log >> $O/workloads.jsonl
  grep '^{' $O/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', r['ms_per_step'], 'analysis_ms', r.get('analysis_ms'))"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload products_bsr16_f16_grp --steps 5 --warmup 2 --no-cpu-baseline) > $O/kt.log 2>&1; rc=$?; stop $rc
timeout -k 10 900 python tools/determinism.py 3 > $O/determinism.log 2>&1; rc=$?; tail -1 $O/determinism.log; stop $rc
exit 0
