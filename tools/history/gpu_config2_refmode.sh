#!/bin/bash
# BASELINE.md §2 row 2, "reference mode": config 2 (ogbn-arxiv stand-in,
# n = 169,343, nnz = 1,166,243, K = 128) dumped as the reference's text CSR
# (tmp/arxiv_indptr.txt / _indices.txt, load_data.cc:125-165), then
# bin/run_csrmm as run_csrmm.cu:46-171 runs it: values 1.0, 10 epochs, no
# warm-up, events on stream 0, "average csrmm cost time". Each impl of the
# reference's CLI; the first run of a fresh process also pays the first
# launch (as the reference's first epoch does).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/config2/tmp
cd gpurun_out/config2
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '$R/spmm-denseblock_amd')
from spmm_hip import prep
rp, ci = prep.powerlaw_csr(169343, 1166243, 13161, 2.3, 1234)
prep.dump_csr('tmp/arxiv', rp, ci)
print('dumped', rp.size - 1, ci.size)
" || exit 1
for spec in "gespmm 0" "cusparseScsrmm 0" "cusparseScsrmm2 1"; do
  echo "== run_csrmm arxiv 128 $spec"
  timeout -k 10 120 $R/spmm-denseblock_amd/bin/run_csrmm arxiv 128 $spec > run_$(echo $spec | tr ' ' _).log 2>&1 || { tail -5 run_*.log; exit 1; }
  grep -E "n=|average|checksum" run_$(echo $spec | tr ' ' _).log
done
