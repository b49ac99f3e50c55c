#!/bin/bash
# Cache-side PMC of the bs 16 fp16 column stream, per variant: L2 hits / misses,
# L1 -> L2 read requests and L1 accesses, TA busy. One pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
BA="--workload products_bsr16_f16 --steps 3 --warmup 1 --no-cpu-baseline"
: > $R/gpurun_out/cs16_cache.txt
for v in ${VARS:-6104 5021}; do
  O=$R/gpurun_out/pmc16c_$v; mkdir -p $O
  i=0
  for group in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr"; do
    i=$((i+1))
    (cd /tmp && SPMM_BSR_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $group -d $O/p$i -o p$i --output-format csv -- python3 $R/bench.py $BA) > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; echo "variant $v pass $i failed"; exit 1; }
  done
  python3 - "$O" "$v" >> $R/gpurun_out/cs16_cache.txt <<'PY'
import csv, glob, sys, collections
o, v = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(o + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bsr16_f16_cs_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(v, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
done
cat $R/gpurun_out/cs16_cache.txt
