#!/usr/bin/env bash
# Bench a list of compile variants: VARIANTS="flagsA|flagsB|..." (each a
# DP_EXTRA_FLAGS string; empty = default build).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu"}
IFS='|' read -ra VS <<< "${VARIANTS:-}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  DP_EXTRA_FLAGS="$v" python -c "import __graft_entry__ as g; g._builder().build(force=True)" > gpurun_out/ab_build_$i.log 2>&1 || exit 3
  timeout -k 10 600 python bench.py $ARGS > gpurun_out/ab_$i.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "variant $i ($v) rc=$rc"; exit $rc; }
  tail -1 gpurun_out/ab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant [$v]', d['value'], 'Mpatch/s', d['kernel_ms_per_launch'], 'ms', 'E', d['E_mean_evals_per_patch'], 'us/eval/CU', round(d['kernel_ms_per_launch']*1e3*256/(d['E_mean_evals_per_patch']*d['config']['batch_per_gpu']),3))"
done
