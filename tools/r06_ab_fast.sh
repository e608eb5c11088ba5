#!/usr/bin/env bash
# A/B of a performance-kernel change on one box: the bit-exact suite on the
# default library, then bench.py's perf_mode alternately on the default library
# and a variant (VARIANT=<file under densepoints_amd/lib/>), REPS times each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_fast_tests.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/ab_fast_tests.log)"; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${REPS:-2}); do
  for lib in libdensepoints.so ${VARIANT:?}; do
    DP_LIB_VARIANT=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-densify --no-seeds \
      --detail gpurun_out/ab_${lib}_$i.json > gpurun_out/ab_${lib}_$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; tail -5 gpurun_out/ab_${lib}_$i.log; exit $rc; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_${lib}_$i.log') if l.startswith('{')][-1])
pm=d.get('perf_mode',{})
print('$lib', 'rep $i', 'value', d['value'], ' '.join('%s=%s'%(k,v.get('Mpatches_per_s')) for k,v in pm.items()))"
  done
done
