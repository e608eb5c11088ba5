#!/usr/bin/env bash
# Parity kernel memory-path counters: translation (UTCL1),
# L1 -> L2 request latency and L2 hit/miss, for the default library and the
# diagnostic build that folds every tap address into 32 MiB
# (libdp_hot32m.so, -DDP_DIAG_HOTIMG).  Output: gpurun_out/tlb/.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
D=gpurun_out/tlb
mkdir -p $D
ARGS="--no-fast --no-densify --no-seeds --no-cpu --steps 2 --warmup 1"
for v in ${VARIANTS:-libdensepoints.so libdp_hot32m.so}; do
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    DP_LIB_VARIANT=$v timeout -s KILL 240 rocprofv3 --pmc $line --kernel-trace --output-format csv \
      -d $D/${v}_p$i -o run -- python3 bench.py $ARGS > $D/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done <<LIST
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
LIST
done
