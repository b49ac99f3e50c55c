set -u
# SQ instruction counters of the bs 2 / 8 grouped small-bs stream on the reddit stand-in (two --pmc passes per workload)
R=$(pwd); export TMPDIR=/tmp; O=$R/gpurun_out/pmc_small; mkdir -p $O
for w in reddit_bsr2 reddit_bsr8; do
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/a_$w -o a --output-format csv -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline) > $O/a_$w.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_SALU SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/b_$w -o b --output-format csv -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline) > $O/b_$w.log 2>&1 || exit $?
done
