#!/bin/bash
# Round-3 second session pass: pytest -m gpu, smoke, the default bench line,
# the hot-column CSR line, and the K = 256 hot probe. Logs in gpurun_out/r03b/.
# A GPU fault, abort or time limit (rc >= 124) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03b; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; stop $rc
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
fi
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-400; stop $rc
for w in ${WLS:-products_csr_hot products_csr}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_$w.log 2>&1; rc=$?; stop $rc
  grep '^{' $O/bw_$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'analysis', r.get('analysis_ms'), 'hot', r.get('hot_gather_share'))"
done
[ -n "${K256:-}" ] && { K=256 HS="0 65536 98304 131072 196608 262144" bash tools/gpu_hot.sh; stop $?; }
exit 0
