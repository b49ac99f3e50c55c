#!/bin/bash
# HBM bytes of each workload's dominant kernel, as MI355X_MICROARCH.md §HBM
# prescribes: a kernel-trace pass for the duration, then FETCH_SIZE and
# WRITE_SIZE in passes of their own (never combined with tracing), plus the
# known-byte calibration run for the FETCH_SIZE correction. Summary lines go
# to gpurun_out/pmcb/bytes.jsonl (tools/bytes_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/pmcb; mkdir -p $O
run() { name=$1; shift; (cd /tmp && timeout -k 10 ${T_STEP:-300} "$@") > $O/$name.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; echo "$name rc=$rc stop"; exit $rc; fi; }
if [ ! -d $O/cfetch ]; then
  run cfetch rocprofv3 --pmc FETCH_SIZE -d $O/cfetch -o cfetch --output-format csv -- python3 $R/tools/pmc_calibrate.py
fi
for wl in ${WLS:-reddit_bsr32 products_bsr32 products_bsr16_f16}; do
  echo "== $wl"
  BA="--workload $wl --no-cpu-baseline ${BENCH_EXTRA:-}"
  run kt_$wl rocprofv3 --kernel-trace --stats -d $O/kt_$wl -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $BA
  grep '^{' $O/kt_$wl.log | cut -c1-160
  run fetch_$wl rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$wl -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $BA
  run write_$wl rocprofv3 --pmc WRITE_SIZE -d $O/write_$wl -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $BA
done
python3 tools/bytes_summary.py $O ${WLS:-reddit_bsr32 products_bsr32 products_bsr16_f16} > $O/bytes.jsonl && cat $O/bytes.jsonl
