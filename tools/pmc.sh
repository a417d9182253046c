#!/bin/bash
# PMC counter passes over a short bench run: one rocprofv3 --pmc pass per counter
# group (never combined with trace domains).  Output: gpurun_out/pmc/<pass>/.
# A pass that fails with an ordinary error (rc 1: e.g. an unknown counter) does
# not stop the script; a timeout, abort or signal does.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${PMC_ARGS:---steps 1 --warmup 1 --no-cpu}
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1
  rc=$?; echo "list rc=$rc"; [ $rc -le 1 ] || exit $rc
fi
run_pass() {
  local name=$1; shift
  timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv \
    -- python bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ $rc -le 1 ] || exit $rc
}
for spec in ${PASSES:-"fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU" "sq2:SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES" "tcc:TCC_HIT_sum,TCC_MISS_sum"}; do
  name=${spec%%:*}
  ctrs=${spec#*:}
  run_pass $name ${ctrs//,/ }
done
