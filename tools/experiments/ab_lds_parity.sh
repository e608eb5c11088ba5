#!/usr/bin/env bash
# Parity-kernel LDS-staging study: the default library and
# the diagnostic variants (DP_DIAG_LDS_PAD / DP_DIAG_LDS_TAPS builds under
# densepoints_amd/lib/), each through bench.py's parity headline only; prints
# rate, E and the time per evaluation.  Alternated twice.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do
for v in ${VARIANTS:-libdensepoints.so}; do
  DP_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --no-fast --no-densify --no-seeds --no-cpu --steps 3 \
    > gpurun_out/abl_${v}_$rep.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abl_${v}_$rep.log; exit $rc; }
  tail -1 gpurun_out/abl_${v}_$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
B=d['config']['batch_per_gpu']
print('$v', 'rep', $rep, 'Mpatches/s', d['value'], 'E', d['E_mean_evals_per_patch'], 'kernel_ms', d['kernel_ms_per_launch'],
      'ns_per_eval', round(d['kernel_ms_per_launch'] * 1e6 / (d['E_mean_evals_per_patch'] * B), 3))"
done
done
