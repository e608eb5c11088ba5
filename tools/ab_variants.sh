#!/usr/bin/env bash
# A/B of prebuilt library variants in one GPU session: VARIANTS="libdensepoints.so libdensepoints_b.so ..."
# (built beforehand with DP_EXTRA_FLAGS and copied under densepoints_amd/lib/), each run
# through the performance-mode tests and bench.py's perf_mode sub-object.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--no-cpu --no-densify --no-seeds --steps 2 --warmup 1"}
for v in ${VARIANTS:-libdensepoints.so}; do
  if [ -n "${TESTS:-}" ]; then
    DP_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest $TESTS -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/ab_test_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/ab_test_$v.log)"
  fi
  DP_LIB_VARIANT=$v timeout -k 10 500 python -u bench.py $ARGS > gpurun_out/ab_$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; exit $rc; }
  tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pm=d['perf_mode']; print('$v', 'parity', d['value'], {k: (v['Mpatches_per_s'], v['kernel_ms_per_launch']) for k, v in pm.items() if isinstance(v, dict) and 'Mpatches_per_s' in v})"
done
