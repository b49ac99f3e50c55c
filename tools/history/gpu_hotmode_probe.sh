#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hm; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_csr_hot.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit $rc; }
for r in 1 2 3; do for m in 1 2; do
  SPMM_CSR_HOT_MODE=$m HS="262144" REPS=30 timeout -k 10 240 python -u tools/csr_hot_probe.py > $O/m${m}_$r.log 2>&1 || exit $?
  echo "mode $m: $(grep '"H": 262144' $O/m${m}_$r.log | head -1 | cut -c1-120) plain $(grep '"H": "plain"' $O/m${m}_$r.log | head -1 | cut -c1-60)"
done; done
