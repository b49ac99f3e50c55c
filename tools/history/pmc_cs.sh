#!/bin/bash
# Issue-side PMC passes for one bs = 32 workload (column-stream kernel):
# instruction mix, per-type active cycles, branch and fetch counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
WL=${WL:-products_bsr32}
O=$R/gpurun_out/pmccs_$WL${TAG:-}
mkdir -p $O
BA="--workload $WL --steps 3 --warmup 1 --no-cpu-baseline"
run() { name=$1; shift; echo "== $name"; (cd /tmp && timeout -k 10 300 "$@") > $O/$name.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; echo "rc=$rc stop"; exit $rc; fi; }
i=0
for group in "SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  run pmc$i rocprofv3 --pmc $group -d $O/pmc$i -o pmc$i --output-format csv -- python3 $R/bench.py $BA
done
python3 tools/pmc_summary.py $O --kernel ${KN:-cs2_kernel} > $O/summary.json && cat $O/summary.json | head -60
