#!/usr/bin/env bash
# One GPU session: rocprofv3 evidence of the given workloads (tools/r04_profile.sh),
# optionally the GPU suite and smoke(), the default bench line, and the 2-rank
# self-launched bench rehearsal on one device (gloo).  Every GPU step has its
# own time limit; any failure stops the script.
#   PROFILE="parity fast7 fast11" TESTS=1 N2=1 bash tools/r04_session.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${PROFILE:-}; do
  bash tools/r04_profile.sh $w || exit $?
done
echo "profiles done"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_final.log; echo; [ $rc -eq 0 ] || exit $rc
fi
if [ "${N2:-0}" = 1 ]; then
  DP_BENCH_ONE_DEVICE=1 DP_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 \
    --no-fast --no-seeds > gpurun_out/bench_n2.log 2>&1
  rc=$?; echo "bench n2 rc=$rc"; tail -c 300 gpurun_out/bench_n2.log; echo; exit $rc
fi
