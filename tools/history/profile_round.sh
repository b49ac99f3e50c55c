#!/bin/bash
# rocprofv3 passes for the bench's dominant kernel: kernel trace + stats, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the bench and for the
# known-byte calibration run. Counters never share a pass with tracing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
O=$R/gpurun_out/prof
mkdir -p $O
BA="${BENCH_ARGS:-} --no-cpu-baseline"
run() { name=$1; shift; echo "== $name"; (cd /tmp && timeout -k 10 400 "$@") > $O/$name.log 2>&1; rc=$?; tail -2 $O/$name.log; if [ $rc -ne 0 ]; then echo "rc=$rc stop"; exit $rc; fi; }
run kt rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $BA
run fetch rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $BA
run write rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $BA
run cfetch rocprofv3 --pmc FETCH_SIZE -d $O/cfetch -o cfetch --output-format csv -- python3 $R/tools/pmc_calibrate.py
run cwrite rocprofv3 --pmc WRITE_SIZE -d $O/cwrite -o cwrite --output-format csv -- python3 $R/tools/pmc_calibrate.py
run hit rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/hit -o hit --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $BA
