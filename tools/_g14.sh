# PMC passes on the headline: LDS / wait / issue counters of the hot kernels
set -u
rm -rf gpurun_out/pmc
PASSES="lds:SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE issue:SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_SMEM" PMC_ARGS="--steps 1 --warmup 1 --no-cpu --no-h2d --no-prof" PASS_TIMEOUT=120 bash tools/pmc.sh
