# PMC SQ counters of the headline's kernels (dense cross-term passes: what bounds them)
set -u
mkdir -p gpurun_out
rm -rf gpurun_out/pmc
PASSES="sq:SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU sq2:SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE fetch:FETCH_SIZE" \
  PMC_ARGS="--steps 2 --warmup 1 --no-cpu --no-h2d --no-prof" PASS_TIMEOUT=120 bash tools/pmc.sh || exit 1
python tools/pmc_table.py gpurun_out/pmc > gpurun_out/pmc_table35.txt 2>&1
grep -i "dn_\|k_tq\b\|k_tp\b\|part_scatter\|sums2" gpurun_out/pmc_table35.txt | head -20
head -3 gpurun_out/pmc_table35.txt
