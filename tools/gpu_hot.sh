#!/bin/bash
# CSR hot-column cache-hint probe (tools/csr_hot_probe.py) over cold-row policies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hot; mkdir -p $O
for a in ${AUXS:-2 1 16 18 3}; do
  echo "== cold aux $a"
  SPMM_CSR_HOT_AUX=$a timeout -k 10 240 python -u tools/csr_hot_probe.py > $O/probe_aux$a.log 2>&1; rc=$?
  grep '^{' $O/probe_aux$a.log | grep -v '"H": "plain"' | head -${NH:-20}; grep plain $O/probe_aux$a.log | head -2
  [ $rc -ge 124 ] && { echo "stop rc=$rc"; exit $rc; }
done
exit 0
