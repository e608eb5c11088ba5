#!/usr/bin/env bash
# Separate --pmc passes (no trace domains besides --kernel-trace) for the
# refine kernel's issue/stall breakdown.  Output: gpurun_out/ctr_<tag>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:-"--steps 1 --warmup 0 --no-cpu --no-densify --no-seeds"}
i=0
mkdir -p gpurun_out/ctr_$TAG
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $line --kernel-trace --output-format csv -d gpurun_out/ctr_$TAG/p$i -o run -- python3 bench.py $ARGS > gpurun_out/ctr_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<LIST
${PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FP64 GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_WAIT_INST_LDS}
LIST
