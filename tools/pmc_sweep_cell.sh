set -u
# SQ counters of the bs 32 column stream on the reference sweep's p = 2e-2 bs 32 cells, dim 64 and
# 128, transB = 1 (two --pmc passes per cell). Output in gpurun_out/pmc_cell/.
R=$(pwd); export TMPDIR=/tmp; O=$R/gpurun_out/pmc_cell; mkdir -p $O
for d in 64 128; do
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/a_$d -o a --output-format csv -- python3 $R/tools/ref_sweep.py --densities 0.02 --bs 32 --dims $d --transB 1 --skip-csr --reps 3) > $O/a_$d.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_SALU SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/b_$d -o b --output-format csv -- python3 $R/tools/ref_sweep.py --densities 0.02 --bs 32 --dims $d --transB 1 --skip-csr --reps 3) > $O/b_$d.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/c_$d -o c --output-format csv -- python3 $R/tools/ref_sweep.py --densities 0.02 --bs 32 --dims $d --transB 1 --skip-csr --reps 3) > $O/c_$d.log 2>&1 || echo "pass c rc=$?"
(cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt_$d -o kt --output-format csv -- python3 $R/tools/ref_sweep.py --densities 0.02 --bs 32 --dims $d --transB 1 --skip-csr --reps 3) > $O/kt_$d.log 2>&1 || exit $?
done
