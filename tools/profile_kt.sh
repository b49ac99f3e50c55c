#!/bin/bash
# rocprofv3 kernel-trace + stats (no counters) for a list of bench workloads;
# summaries land in gpurun_out/kt_<workload>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
for wl in ${WLS:-reddit_bsr32 products_bsr32 products_bsr16_f16 reddit_hybrid32 products_hybrid32}; do
  O=$R/gpurun_out/kt_$wl${KT_TAG:-}; mkdir -p $O
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_EXTRA:-}) > $O/run.log 2>&1 || { tail -5 $O/run.log; echo "kt $wl failed"; exit 1; }
  grep '^{' $O/run.log | cut -c1-200
done
