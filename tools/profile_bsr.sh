#!/bin/bash
# PMC passes for one bench workload (default reddit_bsr32): kernel trace, then
# separate counter passes (SQ stall / MFMA counters, TCC traffic). Counters
# missing from `rocprofv3 -L` on this box are dropped.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
WL=${WL:-reddit_bsr32}
O=$R/gpurun_out/prof_$WL${TAG:-}
mkdir -p $O
(cd /tmp && timeout -k 10 120 rocprofv3 -L) > $O/counters_list.txt 2>&1 || true
have() { grep -qw "$1" $O/counters_list.txt; }
BA="--workload $WL --steps 3 --warmup 1 --no-cpu-baseline ${EXTRA:-}"
run() { name=$1; shift; echo "== $name"; (cd /tmp && timeout -k 10 400 "$@") > $O/$name.log 2>&1; rc=$?; grep '^{' $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; echo "rc=$rc stop"; exit $rc; fi; }
run kt rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py $BA
i=0
for group in ${GROUPS_OVERRIDE:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_EA0_RDREQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr TA_BUSY_max"} ; do
  cs=""; for c in $group; do if have $c; then cs="$cs $c"; fi; done
  i=$((i+1)); [ -z "$cs" ] && continue
  run pmc$i rocprofv3 --pmc $cs -d $O/pmc$i -o pmc$i --output-format csv -- python3 $R/bench.py $BA
done
