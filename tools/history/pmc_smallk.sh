#!/bin/bash
# HBM fetch bytes of the small-K CSR kernel (products stand-in): FETCH_SIZE
# and WRITE_SIZE in separate passes, TCC hit/miss in a third.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
for K in ${KS:-8 32}; do
  O=$R/gpurun_out/pmc_smallk_K$K
  mkdir -p $O
  i=0
  for group in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $group -d $O/p$i -o p$i --output-format csv -- python3 $R/bench.py --K $K --steps 3 --warmup 1 --no-cpu-baseline) > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; echo "pass $i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $O --kernel csr_ > $O/summary.json
  echo "K=$K"; python3 -c "
import json; d=json.load(open('$O/summary.json'))
for k,v in d.items():
    print(' ', k[:60], {c: round(x['mean']) for c,x in v.items() if c!='duration_ns'})"
done
