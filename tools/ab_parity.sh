#!/usr/bin/env bash
# A/B of prebuilt library variants on the parity headline in one GPU session:
# VARIANTS="libdensepoints.so libdensepoints_x.so ..." (built beforehand with
# DP_EXTRA_FLAGS + DP_LIB_NAME); optional TESTS="tests/test_gpu_parity.py" runs
# those tests against each variant first.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--no-cpu --no-densify --no-seeds --no-fast --steps 3 --warmup 1"}
for v in ${VARIANTS:-libdensepoints.so}; do
  if [ -n "${TESTS:-}" ]; then
    DP_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abp_test_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/abp_test_$v.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  fi
  DP_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/abp_$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; exit $rc; }
  tail -1 gpurun_out/abp_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], 'Mpatch/s', d['kernel_ms_per_launch'], 'ms', d.get('stamps_share', ''))"
done
