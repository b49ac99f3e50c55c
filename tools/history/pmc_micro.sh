#!/bin/bash
# PMC passes over tools/bsr_micro.py (MODE=hot): stall and pipe counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp MODE=${MODE:-hot}
O=$R/gpurun_out/pmc_micro_${TAG:-x}
mkdir -p $O
i=0
for group in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU" \
             "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES" \
             "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL" \
             "TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TAGRAM0_REQ TCP_TCC_READ_REQ_sum SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 200 rocprofv3 --pmc $group -d $O/p$i -o p$i --output-format csv -- python3 $R/tools/bsr_micro.py) > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; echo "pass $i failed"; }
done
python3 tools/pmc_summary.py $O --kernel bsr32 > $O/summary.json
python3 - $O/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    print(k[:80])
    for c,x in sorted(v.items()):
        print(f"   {c:36s} {x['mean']:.4g}")
PY
