#!/bin/bash
# Kernel trace of the bs 16 fp16 item stream: builder vs streaming kernel time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
for v in ${VARS:-5533 5522}; do
  O=$R/gpurun_out/kt_is16_$v; mkdir -p $O
  (cd /tmp && SPMM_BSR_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --workload products_bsr16_f16 --steps 10 --warmup 3 --no-cpu-baseline) > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
  f=$(find $O -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('$v', r['Name'][:70], r['Calls'], r['AverageNs'])
" | sort -k4 -n -r | head -6
done
