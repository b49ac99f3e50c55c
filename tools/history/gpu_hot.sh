#!/bin/bash
# CSR hot-column cache-hint probe (tools/csr_hot_probe.py): kernel ms per hot
# budget H (rows) against the plain kernel, C bit-identical. K and HS from the
# environment. (The round-3 sweep over cold-row policies sc0 / sc1 / nt, made
# with a since-removed SPMM_CSR_HOT_AUX knob, is in profiles/r03_hot/.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hot; mkdir -p $O
timeout -k 10 240 python -u tools/csr_hot_probe.py > $O/probe_K${K:-128}.log 2>&1; rc=$?
grep '^{' $O/probe_K${K:-128}.log
exit $rc
