#!/usr/bin/env bash
# End-of-round GPU session: the parity kernel's rocprofv3 evidence
# (tools/r03_profile.sh parity), the whole GPU suite, smoke() and the default
# bench line.  Each GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${PROFILE:-parity}; do
  bash tools/r03_profile.sh $w || exit $?
done
echo "profiles done"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_final.log; exit $rc
